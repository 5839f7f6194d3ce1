#!/usr/bin/env python3
"""Determinism / batch-independence probe: fa_tc_int8_b and fa_tc_int8_pt at the C4 shape, batched twice
and one sequence per call, bitwise comparison (max |diff| and differing-element counts per sequence).
    python tools/det_check.py [--variants fa_tc_int8_pt,fa_tc_int8_b]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizedmha_amd import torch_ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="fa_tc_int8_pt,fa_tc_int8_b")
    ap.add_argument("--rounds", type=int, default=1, help="repeat the single-sequence sweep")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, N, H, d = 16, 4096, 16, 64
    g = torch.Generator(device=dev).manual_seed(4)
    Q = torch.randn(B, N, H * d, device=dev, generator=g) * 0.5
    K = torch.randn(B, N, H * d, device=dev, generator=g) * 0.5
    V = torch.rand(B, N, H * d, device=dev, generator=g)
    for v in a.variants.split(","):
        o1 = torch_ext.flash_solve(Q, K, V, H * d, H, kernel=v)
        o2 = torch_ext.flash_solve(Q, K, V, H * d, H, kernel=v)
        torch.cuda.synchronize()
        print(v, "batched twice: equal", torch.equal(o1, o2), "max", float((o1 - o2).abs().max()), flush=True)
        for b in list(range(B)) * a.rounds:
            one = torch_ext.flash_solve(Q[b], K[b], V[b], H * d, H, kernel=v)
            torch.cuda.synchronize()
            dif = (one - o1[b]).abs()
            nd = int((dif > 0).sum())
            if nd:
                heads = sorted(set(int(c) // d for c in torch.nonzero(dif.amax(0) > 0).flatten().tolist()))
                print(f"  seq {b}: {nd} elements differ, max {float(dif.max()):.3g}, heads {heads}", flush=True)
        print(v, "done", flush=True)


if __name__ == "__main__":
    main()
