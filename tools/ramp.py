#!/usr/bin/env python3
"""Per-call time of the C4 int8 forward over a long run (clock ramp / steady state check)."""
import sys
import os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizedmha_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
B, H, N, d = 16, 16, 4096, 64
g = torch.Generator(device=dev).manual_seed(1)
Q, K, V = (torch.randn(B, N, H * d, device=dev, generator=g) * 0.5 for _ in range(3))
O = torch.empty_like(Q)
lib = _lib.load()
s = torch.cuda.current_stream().cuda_stream
n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
for i in range(n):
    ev[i][0].record()
    lib.qmha_solve_ex(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), B, N, H * d, H, 2, s)
    ev[i][1].record()
torch.cuda.synchronize()
t = [a.elapsed_time(b) for a, b in ev]
for i in range(0, n, 10):
    print(f"calls {i:4d}-{i + 9:4d}: " + " ".join(f"{x:.3f}" for x in t[i:i + 10]))
