#!/usr/bin/env python3
"""Benchmark of the north-star path: fused INT8 attention forward (fa_tc_int8_b) at
BASELINE config 4, B16 H16 N4096 d64 per GPU, through the C-ABI (qmha_solve_ex).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A "step" is one qmha_solve_ex call = one full B x H attention forward (quantisation
pre-pass + fused kernel) with fp32 Q/K/V already resident in HBM.  Multi-GPU: one process
per GPU, each rank owns its own batch shard of 16 sequences (weak scaling, BASELINE
config 5 at N=8), no collective inside the timed region; the RCCL all-gather of the
per-shard outputs named by the north star is timed separately (allgather_ms).
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from quantizedmha_amd import _lib  # noqa: E402

INT8_PEAK_TOPS = 5000.0  # MI355X dense int8 MFMA (2x bf16 2.5 PF; MI355X_MICROARCH.md)
F16_PEAK_TFLOPS = 2500.0
F32_VALU_PEAK_TFLOPS = 157.3
PEAKS = {"fa_tc_int8_b": INT8_PEAK_TOPS, "fa_tc_v1a": F16_PEAK_TFLOPS, "fa": F32_VALU_PEAK_TFLOPS}


def flops(B, H, N, d):
    return 4.0 * B * H * N * N * d  # QK^T 2N^2d + PV 2N^2d per head (softmax excluded)


def run_variant(variant, B, H, N, d, steps, warmup, dev, rank, world, profile=True):
    lib = _lib.load()
    vid = _lib.variant_id(variant)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    Q = torch.randn(B, N, H * d, device=dev, generator=g) * 0.5
    K = torch.randn(B, N, H * d, device=dev, generator=g) * 0.5
    V = torch.randn(B, N, H * d, device=dev, generator=g) * 0.5
    O = torch.empty_like(Q)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    def step():
        st = lib.qmha_solve_ex(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), B, N, H * d, H, vid, sptr)
        _lib.check(st, variant)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    lib.qmha_profile_collect(None, None, None)  # drop anything recorded so far
    lib.qmha_profile_enable(1 if profile else 0)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    lib.qmha_profile_enable(0)
    import ctypes
    main_ms, pre_ms, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_longlong()
    lib.qmha_profile_collect(ctypes.byref(main_ms), ctypes.byref(n), ctypes.byref(pre_ms))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    launches = max(1, n.value)
    return {
        "elapsed_s": elapsed,
        "ms_per_step": elapsed * 1e3 / steps,
        "main_kernel_ms": main_ms.value / launches,
        "prepass_ms": pre_ms.value / launches,
        "launches": n.value,
        "O": O,
    }


def time_solve_calls(variant, B, H, N, d, dev, reps=3):
    """The reference's calling pattern (drivers/main.cu:135-142, torch_ext.cpp:36-40): one
    blocking `solve` per sequence, B of them per step, through the C-ABI (qmha_solve_variant =
    solve with the variant chosen at run time).  Returns ms per B calls."""
    lib = _lib.load()
    vid = _lib.variant_id(variant)
    g = torch.Generator(device=dev).manual_seed(99)
    Q, K, V = (torch.randn(B, N, H * d, device=dev, generator=g) * 0.5 for _ in range(3))
    O = torch.empty_like(Q)
    sz = N * H * d * 4

    def calls():
        for b in range(B):
            st = lib.qmha_solve_variant(Q.data_ptr() + b * sz, K.data_ptr() + b * sz, V.data_ptr() + b * sz,
                                        O.data_ptr() + b * sz, N, H * d, H, vid)
            _lib.check(st, variant)

    calls()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        calls()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) * 1e3 / reps


def time_allgather(O, steps, dev, world):
    out = torch.empty((world,) + tuple(O.shape), dtype=O.dtype, device=dev)
    dist.all_gather_into_tensor(out, O)
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        dist.all_gather_into_tensor(out, O)
    torch.cuda.synchronize(dev)
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()) * 1e3 / steps


def cpu_baseline(budget_s=20.0):
    """The reference's CPU verify path (utils/verify.cu cpu_reference, compiled from the
    reference sources into oracle/_ref) timed on this host, 1 thread, on a bounded sample:
    B1 H4 N2048 d64 (RoPE included, as in the reference)."""
    from oracle import oracle
    kind = "reference"
    fn = None
    try:
        if oracle.ref_lib() is not None:
            fn = oracle.ref_cpu_reference
    except Exception:
        fn = None
    if fn is None:
        kind = "port"
        fn = oracle.cpu_reference_rope
    rng = np.random.default_rng(42)
    N, H, d = 2048, 4, 64
    Q, K, V = (rng.random((N, H * d), dtype=np.float32) for _ in range(3))
    # size the sample to the budget: time one head first
    t0 = time.perf_counter()
    devnull = os.open(os.devnull, os.O_WRONLY)
    saved = os.dup(1)
    os.dup2(devnull, 1)  # cpu_reference prints a progress bar
    try:
        fn(Q[:, :d], K[:, :d], V[:, :d], d, 1)
        t_head = time.perf_counter() - t0
        heads = int(max(1, min(H, budget_s // max(t_head, 1e-3))))
        t0 = time.perf_counter()
        fn(Q[:, :heads * d], K[:, :heads * d], V[:, :heads * d], heads * d, heads)
        t = time.perf_counter() - t0
    finally:
        os.dup2(saved, 1)
        os.close(saved)
        os.close(devnull)
    value = flops(1, heads, N, d) / t / 1e12
    res = {"value": value, "unit": "TFLOPS", "cores": 1, "kind": kind,
           "sample": f"utils/verify.cu cpu_reference (RoPE) B1 H{heads} N{N} d{d}, 1 thread, {t:.2f} s; "
                     f"attention-equivalent 4*H*N^2*d FLOPs", "seconds": round(t, 3),
           "host_cpu": _cpu_model(), "nproc": os.cpu_count()}
    res["port_int8"] = cpu_port_int8()
    return res


def cpu_port_int8(threads=16, N=4096, H=16, d=64):
    """The same int8 algorithm as the GPU path (oracle/qmha_oracle.c oracle_fa_int8, the CPU
    restatement of fa_tc_int8_b), multi-threaded over heads on `threads` host cores (the
    GPU box's CPU share), on one sequence of the C4 shape: the practical CPU verify path."""
    from oracle import oracle
    threads = max(1, min(threads, os.cpu_count() or 1))
    rng = np.random.default_rng(7)
    Q, K, V = (rng.standard_normal((N, H * d), dtype=np.float32) * 0.5 for _ in range(3))
    t0 = time.perf_counter()
    oracle.fa_int8(Q, K, V, H * d, H, nthreads=threads)
    t = time.perf_counter() - t0
    return {"value": flops(1, H, N, d) / t / 1e12, "unit": "TFLOPS", "cores": threads, "kind": "port",
            "sample": f"oracle_fa_int8 B1 H{H} N{N} d{d} (one sequence of the C4 workload), "
                      f"{threads} threads, {t:.2f} s", "seconds": round(t, 3)}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc_traffic(variant, B, H, N, d):
    """HBM bytes per main-kernel launch from the committed rocprofv3 PMC summary
    (profiles/*/pmc_<variant>.json, produced by tools/pmc_summary.py), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", f"pmc_{variant}.json")), reverse=True):
        try:
            j = json.load(open(path))
            if j.get("shape") == [B, H, N, d]:
                return j.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
        except Exception:
            continue
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--variant", default="fa_tc_int8_b", choices=list(_lib.VARIANTS))
    ap.add_argument("--B", type=int, default=16, help="sequences per GPU")
    ap.add_argument("--H", type=int, default=16)
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--no-siblings", action="store_true", help="skip the fp16 / fp32 sibling measurements")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-solve-calls", action="store_true",
                    help="skip the one-solve-per-sequence timing (profiled runs: keeps its B=1 launches "
                         "out of the main kernel's rocprof average)")
    ap.add_argument("--allgather", action="store_true", default=None,
                    help="time the RCCL all-gather of per-shard outputs (default on when N>1)")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    B, H, N, d = a.B, a.H, a.N, a.d

    r = run_variant(a.variant, B, H, N, d, a.steps, a.warmup, dev, rank, world)
    total_flops = flops(B, H, N, d) * world
    value = total_flops / r["elapsed_s"] * a.steps / 1e12
    peak = PEAKS.get(a.variant, INT8_PEAK_TOPS)
    achieved = flops(B, H, N, d) / (r["main_kernel_ms"] * 1e-3) / 1e12
    traffic, traffic_src = pmc_traffic(a.variant, B, H, N, d)
    hbm_alg = 16.0 * B * N * H * d  # fp32 Q, K, V read once + O written once (per call)
    res = {
        "metric": "attention-fwd TFLOPS + ms/call, B16 H16 N4096 d64 (fp16 & int8)",
        "value": round(value, 3),
        "unit": "TFLOPS",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(r["ms_per_step"], 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8" if a.variant == "fa_tc_int8_b" else ("fp16" if a.variant == "fa_tc_v1a" else "fp32"),
        "data": "synthetic N(0, 0.5^2) fp32 Q/K/V, torch.Generator seed 1234+rank, resident in HBM",
        "config": {"workload": f"{a.variant} attention forward (BASELINE config 4{'/5' if world > 1 else ''})",
                   "variant": a.variant, "B_per_gpu": B, "H": H, "N": N, "d": d, "d_model": H * d,
                   "global_batch": B * world, "parallelism": f"batch-shard x{world} (no collective in step)"},
        "roofline": {"bound": "mfma", "kernel": f"qmha_fa_{'int8' if a.variant == 'fa_tc_int8_b' else a.variant}",
                     "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "algorithmic_flops_per_launch": flops(B, H, N, d),
                     "main_kernel_ms": round(r["main_kernel_ms"], 4),
                     "prepass_ms": round(r["prepass_ms"], 4),
                     "hbm_algorithmic_bytes_per_call": hbm_alg},
    }
    if world > 1 and a.allgather is not False:
        ag_ms = time_allgather(r["O"], max(3, a.steps // 2), dev, world)
        res["allgather_ms"] = round(ag_ms, 4)
        res["value_with_allgather"] = round(total_flops / ((r["ms_per_step"] + ag_ms) * 1e-3) / 1e12, 3)
    del r
    if not a.no_siblings:
        sib = {}
        for v in ("fa_tc_v1a", "fa"):
            Bs = B if v != "fa" else 8
            Hs = H if v != "fa" else 8
            Ns = N if v != "fa" else 1024
            rv = run_variant(v, Bs, Hs, Ns, d, max(3, a.steps // 2), 2, dev, rank, world)
            sib[v] = {"config": f"B{Bs} H{Hs} N{Ns} d{d}", "ms_per_step": round(rv["ms_per_step"], 4),
                      "tflops": round(flops(Bs, Hs, Ns, d) * world / (rv["ms_per_step"] * 1e-3) / 1e12, 3),
                      "main_kernel_ms": round(rv["main_kernel_ms"], 4),
                      "roofline_frac": round(flops(Bs, Hs, Ns, d) / (rv["main_kernel_ms"] * 1e-3) / 1e12 /
                                             PEAKS[v], 4)}
            del rv
        res["siblings"] = sib
    if rank == 0 and world == 1 and not a.no_siblings and not a.no_solve_calls:
        ms = time_solve_calls(a.variant, B, H, N, d, dev)
        res["solve_calls"] = {"pattern": f"{B} blocking solve() calls, one per sequence (reference usage)",
                              "ms_per_step": round(ms, 4), "tflops": round(flops(B, H, N, d) / (ms * 1e-3) / 1e12, 3)}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
