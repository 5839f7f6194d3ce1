#!/usr/bin/env python3
"""Where the reference's one-sequence-per-call pattern loses time.

Runs, back to back, each as a labelled burst (hipEvents on the stream + wall clock):
  batched   one qmha_solve_ex over B sequences (the headline call)
  async1    B qmha_solve_ex calls of one sequence each, no synchronisation (torch_ext's pattern)
  solve     B blocking qmha_solve_variant calls (solve()'s pattern: null stream + sync per call)
  refB      the reference's own shape (B1..B4 H32 N8192 d32) batched, per-sequence time
Run it under `rocprofv3 --kernel-trace` to split each burst into per-dispatch kernel durations and
the gaps between dispatches (tools/probe_split.py reads the trace).
    python tools/probe_calls.py [--reps 5] [--variant fa_tc_int8_b]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizedmha_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variant", default="fa_tc_int8_b")
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--H", type=int, default=16)
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--bursts", default="batched,async1,solve,batched_again,ref",
                    help="comma-separated subset of batched, async1, solve, batched_again, ref")
    a = ap.parse_args()
    lib = _lib.load()
    if os.environ.get("QMHA_OVERLAP"):  # batch chunks with the pre-pass of chunk c+1 beside chunk c's main kernel
        lib.qmha_set_overlap_chunks(int(os.environ["QMHA_OVERLAP"]))
    vid = _lib.variant_id(a.variant)
    dev = torch.device("cuda:0")
    B, H, N, d = a.B, a.H, a.N, a.d
    g = torch.Generator(device=dev).manual_seed(5)
    Q, K, V = (torch.randn(B, N, H * d, device=dev, generator=g) * 0.5 for _ in range(3))
    O = torch.empty_like(Q)
    s = torch.cuda.current_stream(dev)
    sp = s.cuda_stream
    sz = N * H * d * 4
    res = {}

    def burst(name, fn, reps):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3 / reps
        res[name] = {"wall_ms": round(wall, 4), "event_ms": round(e0.elapsed_time(e1) / reps, 4)}
        print(name, res[name], flush=True)

    def batched():
        _lib.check(lib.qmha_solve_ex(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), B, N, H * d, H, vid, sp))

    def async1():
        for b in range(B):
            _lib.check(lib.qmha_solve_ex(Q.data_ptr() + b * sz, K.data_ptr() + b * sz, V.data_ptr() + b * sz,
                                         O.data_ptr() + b * sz, 1, N, H * d, H, vid, sp))

    def solve_calls():
        for b in range(B):
            _lib.check(lib.qmha_solve_variant(Q.data_ptr() + b * sz, K.data_ptr() + b * sz, V.data_ptr() + b * sz,
                                              O.data_ptr() + b * sz, N, H * d, H, vid))

    sel = set(a.bursts.split(","))
    for _ in range(20):  # clock ramp
        batched()
    for name, fn in (("batched", batched), ("async1", async1), ("solve", solve_calls), ("batched_again", batched)):
        if name in sel:
            burst(name, fn, a.reps)
    if "ref" not in sel:
        print(json.dumps(res))
        return
    # the reference's own shape at B = 1, 2, 4 (per-sequence throughput vs grid fill)
    del Q, K, V, O
    for Bn in (1, 2, 4):
        Nr, Hr, dr = 8192, 32, 32
        Qr, Kr, Vr = (torch.rand(Bn, Nr, Hr * dr, device=dev, generator=g) for _ in range(3))
        Or = torch.empty_like(Qr)

        def ref_b():
            _lib.check(lib.qmha_solve_ex(Qr.data_ptr(), Kr.data_ptr(), Vr.data_ptr(), Or.data_ptr(), Bn, Nr, Hr * dr, Hr,
                                         vid, sp))
        for _ in range(5):
            ref_b()
        burst(f"ref_B{Bn}", ref_b, a.reps)
        del Qr, Kr, Vr, Or
    print(json.dumps(res))


if __name__ == "__main__":
    main()
