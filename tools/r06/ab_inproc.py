#!/usr/bin/env python3
"""Same-process, alternating A/B of two or more builds of libqmha.so (r06).

Every library is loaded into ONE process (ctypes, different paths: separate code objects and workspaces),
and the rounds alternate A, B, A, B ... on the same inputs, so box, clock and thermal state are shared.
Per round and library: W warm-up calls, then K timed calls with the library's own hipEvent profiling of
its main kernel and pre-pass (qmha_profile_enable / qmha_profile_collect) and host wall time per call.
Outputs are compared bit for bit between the libraries.

    python tools/r06/ab_inproc.py --libs base=quantizedmha_amd/alt_lib/r06base/libqmha.so,new=quantizedmha_amd/lib/libqmha.so \\
        --variants fa_tc_v1a,fa_tc_int8_pt --rounds 4
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from quantizedmha_amd import _lib  # noqa: E402


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    for name in ("qmha_solve_ex", "qmha_profile_enable", "qmha_profile_collect", "qmha_last_error"):
        res, args = _lib.SIGNATURES[name]
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--variants", default="fa_tc_int8_b")
    ap.add_argument("--shape", default="16,4096,16,64", help="B,N,H,d")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    a = ap.parse_args()
    libs = [(n, load(p)) for n, p in (x.split("=", 1) for x in a.libs.split(","))]
    B, N, H, d = (int(x) for x in a.shape.split(","))
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev).manual_seed(1234)
    Q, K, V = (torch.randn(B, N, H * d, device=dev, generator=g) * 0.5 for _ in range(3))
    flops = 4.0 * B * H * N * N * d
    res = {}
    for v in a.variants.split(","):
        vid = _lib.variant_id(v)
        outs = {}
        for n, lib in libs:  # first call of each: outputs for the bit-identity check, and the clock ramp
            O = torch.full_like(Q, float("nan"))
            for _ in range(a.warmup):
                assert lib.qmha_solve_ex(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), B, N, H * d, H, vid, s) == 0
            torch.cuda.synchronize()
            outs[n] = O
        same = {n: torch.equal(outs[libs[0][0]], outs[n]) for n, _ in libs[1:]}
        rows = {n: [] for n, _ in libs}
        for r in range(a.rounds):
            order = libs if r % 2 == 0 else libs[::-1]
            for n, lib in order:
                O = outs[n]
                for _ in range(a.warmup):
                    lib.qmha_solve_ex(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), B, N, H * d, H, vid, s)
                torch.cuda.synchronize()
                lib.qmha_profile_collect(None, None, None)
                lib.qmha_profile_enable(1)
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    lib.qmha_solve_ex(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), B, N, H * d, H, vid, s)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                lib.qmha_profile_enable(0)
                mm, pm, cnt = ctypes.c_double(), ctypes.c_double(), ctypes.c_longlong()
                lib.qmha_profile_collect(ctypes.byref(mm), ctypes.byref(cnt), ctypes.byref(pm))
                k = max(1, cnt.value)
                rows[n].append({"call_ms": (t1 - t0) * 1e3 / a.steps, "main_ms": mm.value / k, "pre_ms": pm.value / k})
        summ = {}
        for n, rr in rows.items():
            mains = [x["main_ms"] for x in rr]
            calls = [x["call_ms"] for x in rr]
            summ[n] = {"main_ms_rounds": [round(x, 4) for x in mains], "call_ms_rounds": [round(x, 4) for x in calls],
                       "main_ms_mean": round(sum(mains) / len(mains), 4), "call_ms_mean": round(sum(calls) / len(calls), 4),
                       "pre_ms_mean": round(sum(x["pre_ms"] for x in rr) / len(rr), 4),
                       "tflops_main": round(flops / (sum(mains) / len(mains) * 1e-3) / 1e12, 1)}
        base = summ[libs[0][0]]["main_ms_mean"]
        for n in summ:
            summ[n]["main_vs_first"] = round(summ[n]["main_ms_mean"] / base - 1.0, 4)
        res[v] = {"shape": [B, N, H, d], "bit_identical_to_first": same, "libs": summ}
        print(v, json.dumps(res[v]), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
