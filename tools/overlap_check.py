#!/usr/bin/env python3
"""Chunked pre-pass/main overlap must be bit-identical to the unchunked call: run the same
inputs with 1 and 4 overlap chunks (qmha_set_overlap_chunks, set inside each child: the
QMHA_OVERLAP_CHUNKS variable is read by QMHA_ABLATION builds only) in two subprocesses and
compare.  Each child checks that the library accepted its chunk count."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(B, N, H, d, variant, chunks, out):
    import torch
    sys.path.insert(0, ROOT)
    from quantizedmha_amd import _lib, torch_ext
    lib = _lib.load()
    lib.qmha_set_overlap_chunks(chunks)
    assert lib.qmha_set_overlap_chunks(chunks) == chunks, "overlap chunk count not applied"
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    Q, K, V = (torch.randn(B, N, H * d, device=dev, generator=g) * 0.5 for _ in range(3))
    o = torch_ext.flash_solve(Q, K, V, H * d, H, kernel=variant)
    o2 = torch_ext.flash_solve(Q, K, V, H * d, H, kernel=variant)  # a second call reuses the workspace
    torch.cuda.synchronize()
    np.save(out, np.stack([o.cpu().numpy(), o2.cpu().numpy()]))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child(*map(int, sys.argv[2:6]), sys.argv[6], int(sys.argv[7]), sys.argv[8])
        sys.exit(0)
    bad = 0
    shapes = ((16, 1024, 16, 64), (8, 512, 4, 64), (3, 256, 2, 128))
    if os.environ.get("OVL_SHAPES"):
        shapes = [tuple(map(int, x.split("x"))) for x in os.environ["OVL_SHAPES"].split()]
    for variant in os.environ.get("OVL_VARIANTS", "fa_tc_int8_b fa_tc_v1a").split():
        for B, N, H, d in shapes:
            res = []
            for chunks in (1, 4):
                out = f"/tmp/ovl_{variant}_{B}_{chunks}.npy"
                subprocess.run([sys.executable, __file__, "child", str(B), str(N), str(H), str(d), variant,
                                str(chunks), out], check=True)
                res.append(np.load(out))
            same = np.array_equal(res[0], res[1])
            diff = float(np.abs(res[0] - res[1]).max())
            rows = np.where(np.abs(res[0] - res[1]).reshape(2, B, -1).max(axis=2) > 0)
            print(variant, (B, N, H, d), "identical" if same else f"DIFF max {diff:.3e} (call, batch) {list(zip(*rows))[:8]}")
            bad += not same
    sys.exit(1 if bad else 0)
