#!/usr/bin/env python3
"""Bit-identity of two builds of libqmha.so on the same inputs (A/B kernels that must not change results).
    python tools/r05/cmp_libs.py <libA.so> <libB.so> [variant]"""
import ctypes
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from quantizedmha_amd import _lib  # noqa: E402


def load(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    return lib


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    vid = _lib.variant_id(sys.argv[3] if len(sys.argv) > 3 else "fa_tc_int8_b")
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    bad = 0
    for (B, N, H, d) in [(16, 4096, 16, 64), (1, 4096, 16, 64), (2, 1024, 8, 64), (3, 2080, 3, 64), (1, 8192, 32, 32),
                         (2, 2048, 4, 128), (2, 96, 2, 64)]:
        g = torch.Generator(device=dev).manual_seed(B * N + d)
        Q, K, V = (torch.randn(B, N, H * d, device=dev, generator=g) * 0.5 for _ in range(3))
        outs = []
        for lib in (a, b):
            O = torch.full_like(Q, float("nan"))
            st = lib.qmha_solve_ex(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), B, N, H * d, H, vid, s)
            assert st == 0, lib.qmha_last_error()
            torch.cuda.synchronize()
            outs.append(O)
        same = torch.equal(outs[0], outs[1])
        bad += not same
        print(f"B{B} N{N} H{H} d{d}: {'bit-identical' if same else 'DIFFERENT max %.3g' % (outs[0] - outs[1]).abs().max().item()}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
