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
import re
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from quantizedmha_amd import _lib  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
INT8_PEAK_TOPS = 5000.0  # MI355X dense int8 MFMA (2x bf16 2.5 PF; MI355X_MICROARCH.md)
F16_PEAK_TFLOPS = 2500.0
F32_VALU_PEAK_TFLOPS = 157.3
F32_MFMA_PEAK_TFLOPS = 157.3  # v_mfma_f32_32x32x2_f32 runs at the fp32 vector rate (MI355X_MICROARCH.md)
PEAKS = {"fa_tc_int8_b": INT8_PEAK_TOPS, "fa_tc_v1a": F16_PEAK_TFLOPS, "fa": F32_VALU_PEAK_TFLOPS,
         "fa_mfma": F32_MFMA_PEAK_TFLOPS, "unfused": F32_VALU_PEAK_TFLOPS, "fa_tc_int8_pt": INT8_PEAK_TOPS}
PEAK_KIND = {"fa_tc_int8_b": "int8 MFMA", "fa_tc_v1a": "f16 MFMA", "fa": "fp32 VALU (no matrix cores)",
             "fa_mfma": "fp32 MFMA", "unfused": "fp32 MFMA GEMMs", "fa_tc_int8_pt": "int8 MFMA"}


def flops(B, H, N, d):
    return 4.0 * B * H * N * N * d  # QK^T 2N^2d + PV 2N^2d per head (softmax excluded)


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def max_over_ranks(x, dev):
    """MAX of a host float over all ranks (the slowest rank defines the step)."""
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class SysfsSampler:
    """Samples this GPU's hwmon clock and power (sysfs file reads on a host thread, no GPU calls) every
    `period` seconds while the timed calls run: the clock the main kernel actually ran at, beside the
    in-kernel probe's (round-5 VERDICT item 2)."""

    def __init__(self, hwmon, period=0.002):
        self.files = {k: os.path.join(hwmon, f) for k, f in (("sclk_mhz", "freq1_input"), ("power_w", "power1_input"))
                      if hwmon and os.path.exists(os.path.join(hwmon, f))}
        self.period, self.samples, self._stop = period, {k: [] for k in self.files}, None

    def __enter__(self):
        import threading
        self._stop = threading.Event()

        def loop():
            while not self._stop.is_set():
                for k, path in self.files.items():
                    v = _read(path)
                    if v and v.isdigit():
                        self.samples[k].append(int(v) * 1e-6)
                self._stop.wait(self.period)
        self._t = threading.Thread(target=loop, daemon=True)
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._t.join()

    def summary(self):
        out = {}
        for k, v in self.samples.items():
            if v:
                out[k] = {"mean": round(sum(v) / len(v), 1), "min": round(min(v), 1), "max": round(max(v), 1), "n": len(v)}
        return out


def run_variant(variant, B, H, N, d, steps, warmup, dev, rank, world, profile=True, dry_run=False, uniform=False,
                sampler=None):
    """Time `steps` qmha_solve_ex calls on this rank's own shard (B sequences), bracketed by a
    barrier + device synchronisation on both sides; the max over ranks is returned.
    dry_run (CPU, gloo; launcher/rendezvous plumbing only): the step is a tensor copy.
    Inputs N(0, 0.5^2) (the reference's golden distribution, tests/generate_golden.cpp); uniform: U[0, 1)
    (its profiling distribution, inputs/data.cu:16-22) -- the kernels' arithmetic does not depend on the
    data, but the chip's clock does (it is power-limited under this kernel)."""
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    if uniform:
        Q, K, V = (torch.rand(B, N, H * d, device=dev, generator=g) for _ in range(3))
    else:
        Q = torch.randn(B, N, H * d, device=dev, generator=g) * 0.5
        K = torch.randn(B, N, H * d, device=dev, generator=g) * 0.5
        V = torch.randn(B, N, H * d, device=dev, generator=g) * 0.5
    O = torch.empty_like(Q)
    if dry_run:
        lib = None

        def step():
            O.copy_(Q)
    else:
        lib = _lib.load()
        vid = _lib.variant_id(variant)
        sptr = torch.cuda.current_stream(dev).cuda_stream

        def step():
            st = lib.qmha_solve_ex(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), B, N, H * d, H, vid, sptr)
            _lib.check(st, variant)

    for _ in range(warmup):
        step()
    _sync(dev)
    if lib is not None:
        lib.qmha_profile_collect(None, None, None)  # drop anything recorded so far
        lib.qmha_profile_enable(1 if profile else 0)
    if dist.is_initialized():
        dist.barrier()
    _sync(dev)
    import contextlib
    with (sampler or contextlib.nullcontext()):
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        _sync(dev)
        t1 = time.perf_counter()
    if dist.is_initialized():
        dist.barrier()
    elapsed = max_over_ranks(t1 - t0, dev)
    import ctypes
    main_ms, pre_ms, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_longlong()
    if lib is not None:
        lib.qmha_profile_enable(0)
        lib.qmha_profile_collect(ctypes.byref(main_ms), ctypes.byref(n), ctypes.byref(pre_ms))
    launches = max(1, n.value)
    return {
        "elapsed_s": elapsed,
        "ms_per_step": elapsed * 1e3 / steps,
        "main_kernel_ms": main_ms.value / launches,
        "prepass_ms": pre_ms.value / launches,
        "launches": n.value,
        "inputs": (Q, K, V),
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
    """The RCCL all-gather of every rank's output shard alone (ms per gather, max over ranks)."""
    out = torch.empty((world * O.shape[0],) + tuple(O.shape[1:]), dtype=O.dtype, device=dev)
    dist.all_gather_into_tensor(out, O)
    _sync(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        dist.all_gather_into_tensor(out, O)
    _sync(dev)
    dist.barrier()
    return max_over_ranks(time.perf_counter() - t0, dev) * 1e3 / steps


def time_solve_gather(variant, inputs, H, d, steps, dev, world, chunks, dry_run=False):
    """Compute + gather per step (shard.solve_shard_gather): each rank's kernels write into its
    slab of the [world * B, N, d_model] result, and chunk c's point-to-point exchange with every
    peer overlaps the compute of chunk c+1; ms per step, max over ranks."""
    from quantizedmha_amd.shard import solve_shard_gather
    Q, K, V = inputs
    batch = Q.shape[0] * world  # every rank holds an equal shard here
    fn = (lambda q, k, v, dm, h, kern: q.clone()) if dry_run else None
    out = Q.new_empty((batch,) + tuple(Q.shape[1:]))

    def step():
        return solve_shard_gather(Q, K, V, H * d, H, batch, variant, chunks=chunks, solve_fn=fn, out=out)

    out = step()
    _sync(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    _sync(dev)
    dist.barrier()
    ms = max_over_ranks(time.perf_counter() - t0, dev) * 1e3 / steps
    assert out.shape[0] == batch
    return ms


def cpu_baseline(budget_s=15.0):
    """The reference's CPU verify path (utils/verify.cu cpu_reference, compiled from the
    reference sources into oracle/_ref) timed on this host, 1 thread, on a bounded sample:
    B1 N2048 d64 with as many of the C4 workload's 16 heads as fit ~15 s (RoPE included, as in
    the reference)."""
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
    N, H, d = 2048, 16, 64
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


def clock_probe(dev):
    """The shader clock under an MFMA + VALU mix like the int8 main kernel's (libqmha_probe.so,
    quantizedmha_amd/csrc/qmha_clock_probe.hip: s_memtime cycles / s_memrealtime ticks, in-kernel), run right
    after the headline so it sees the same thermal / power state."""
    import ctypes
    path = os.path.join(ROOT, "quantizedmha_amd", "lib", "libqmha_probe.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.qmha_clock_probe.restype = ctypes.c_int
    lib.qmha_clock_probe.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    out = (ctypes.c_double * 4)()
    st = lib.qmha_clock_probe(5, 20, out)
    torch.cuda.synchronize(dev)
    if st != 0:
        return {"error": f"hip error {st}"}
    return {"clock_ghz": round(out[0], 4), "ns_per_unit_per_simd": round(out[1], 3),
            "cycles_per_unit": round(out[2], 2), "timed_ms": round(out[3], 3),
            "unit": "1 v_mfma_i32_32x32x32_i8 + 3 v_exp_f32 + 21 v_fma_f32, 3 waves/SIMD"}


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def device_state(dev):
    """This GPU's power cap and power draw from sysfs (hwmon of its PCI function; plain file reads, no
    rocm-smi), plus the identity torch reports."""
    import glob
    p = torch.cuda.get_device_properties(dev)
    out = {"name": p.name, "arch": getattr(p, "gcnArchName", None), "cus": p.multi_processor_count}
    dom, bus, devn = (getattr(p, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    hw = []
    if bus is not None:
        pci = f"{dom or 0:04x}:{bus:02x}:{devn or 0:02x}.0"
        out["pci"] = pci
        hw = glob.glob(f"/sys/bus/pci/devices/{pci}/hwmon/hwmon*")
    if hw:
        h = hw[0]
        for key, fn, scale in (("power_cap_w", "power1_cap", 1e-6), ("power_cap_max_w", "power1_cap_max", 1e-6),
                               ("power_now_w", "power1_average", 1e-6), ("power_input_w", "power1_input", 1e-6),
                               ("sclk_mhz", "freq1_input", 1e-6), ("temp_edge_c", "temp1_input", 1e-3),
                               ("temp_hotspot_c", "temp2_input", 1e-3)):
            v = _read(os.path.join(h, fn))
            if v is not None and v.lstrip("-").isdigit():
                out[key] = round(int(v) * scale, 1)
        out["hwmon"] = h
    return out


def isa_ids(variant, d):
    """isa_sha16 of the shipped main kernel and pre-pass of this variant at head size d: the first 16 hex
    digits of the SHA-256 of their gfx950 instruction bytes in the loaded libqmha.so (quantizedmha_amd/isa_id.py)."""
    from quantizedmha_amd import isa_id
    pats = {"fa_tc_int8_b": (f"qmha_fa_int8_pipe_kernelILi{d}E", f"qmha_quant_int8_kernelILi{d}ELi1E"),
            "fa_tc_int8_pt": (f"qmha_fa_int8_pt_v3_kernelILi{d}ELi8ELi2ELb0E" if d == 64 else f"qmha_fa_int8_pipe_kernelILi{d}E",
                              f"qmha_pt_quant_kernelILi{d}E"),
            "fa_tc_v1a": (f"qmha_fa_f16_{'v3' if d in (64, 128) else 'v2'}_kernelILi{d}E", f"qmha_convert_f16_kernelILi{d}E"),
            "fa": (f"qmha_fa_f32_v3_kernelILi{d}E", None), "fa_mfma": (f"qmha_fa_f32_mfma_kernelILi{d}E", None),
            "unfused": ("qmha_gemm_f32_mfma_kernel", "qmha_softmax_rows")}.get(variant, (None, None))
    out = {}
    for role, pat in zip(("main", "prepass"), pats):
        if not pat:
            continue
        ks = isa_id.kernel_bytes(_lib.LIB_PATH, pat)
        if variant.startswith("fa_tc_int8"):  # the production instance: FL_DUMP (256) clear, FL_PT (1 << 20) as the variant
            want_pt = variant == "fa_tc_int8_pt"
            keep = {}
            for name, b in ks.items():
                fl = re.search(r"ILi\d+ELi\d+ELi(\d+)E", name)
                if role == "main" and "pipe_kernel" in name and fl and (int(fl.group(1)) & 256 or bool(int(fl.group(1)) & (1 << 20)) != want_pt):
                    continue
                keep[name] = b
            ks = keep
        if ks:
            name = sorted(ks)[0]
            import hashlib
            out[role] = {"isa_sha16": hashlib.sha256(b"".join(ks[k] for k in sorted(ks))).hexdigest()[:16],
                         "symbols": len(ks), "bytes": sum(len(b) for b in ks.values()), "symbol": name}
    return out


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


def pmc_sq(variant, B, H, N, d):
    """MFMA-busy % of the main kernel from the committed SQ counter passes
    (profiles/*/pmc_sq_<variant>.json, tools/pmc_sq.sh): the rocprofv3 cross-check SURVEY 8(d) asks for."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", f"pmc_sq_{variant}.json")), reverse=True):
        try:
            j = json.load(open(path))
            if j.get("shape") == [B, H, N, d]:
                return j.get("mfma_busy_pct"), os.path.relpath(path, ROOT)
        except Exception:
            continue
    return None, None


def spawn_ranks(n):
    """`--gpus N` (N > 1) outside a torch.distributed launcher: start the N rank processes (one
    per GPU, rendezvous on 127.0.0.1) with torch.distributed.run as a CHILD process and return
    its exit status.  Nothing in this parent process has touched the GPU (no HIP call, no
    torch.cuda query), so the ranks own their devices from a clean state."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL)
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    # 30 warm-up calls: the clock ramps for the first ~20-30 back-to-back calls of a fresh process
    # (per-call times 1.8 -> 1.47 ms on one box, tools/ramp.py -> profiles/r02/clock_ramp.txt)
    ap.add_argument("--warmup", type=int, default=30)
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
    ap.add_argument("--no-refconfig", action="store_true",
                    help="skip the reference's own configuration (include/config.h: N8192 d_model1024 h32)")
    ap.add_argument("--gather-chunks", type=int, default=4,
                    help="batch chunks of the compute+all-gather step (gather of chunk c overlaps chunk c+1)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher plumbing only (CPU, gloo): spawn, rendezvous, barriers, max-over-ranks "
                         "timing and the chunked all-gather, with a tensor copy as the step; no kernel, no value")
    a = ap.parse_args()

    launched = "WORLD_SIZE" in os.environ
    if not launched and a.gpus > 1:
        sys.exit(spawn_ranks(a.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        sys.stderr.write(f"bench.py: --gpus {a.gpus} but the launcher started {world} ranks\n")
        sys.exit(2)
    dry = a.dry_run
    if dry:
        dev = torch.device("cpu")
        B, H, N, d = min(a.B, 4), min(a.H, 2), min(a.N, 128), a.d
    else:
        if not torch.cuda.is_available():
            sys.stderr.write("bench.py: no GPU visible (the HIP kernels have no CPU path); --dry-run tests the launcher\n")
            sys.exit(2)
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)
        B, H, N, d = a.B, a.H, a.N, a.d
    if launched:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if dry:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    # The side measurements run BEFORE the headline: they are independent of it, and they bring
    # the GPU out of its idle clock state, so the headline's W warm-up calls start from a busy
    # GPU (a fresh process otherwise ramps over its first ~20-30 calls, tools/ramp.py ->
    # profiles/r02/clock_ramp.txt).  The headline itself is still W untimed + K timed calls.
    side = {}
    if not a.no_siblings and not dry:
        sib = {}
        # fa_tc_v1a at C3 (= the C4 shape), fa (the scalar no-matrix-core kernel BASELINE C2 names)
        # and its fp32-MFMA sibling fa_mfma at C2, and the reference's unfused 3-kernel baseline
        # (README.md:11, the fused-vs-unfused comparison) at the C4 shape
        # fa_tc_int8_pt: the per-tensor int8 mode (BASELINE.json's "per-tensor Q/K/V quant" wording;
        # not the reference's per-block numerics, so never the headline) at the C4 shape
        for v in ("fa_tc_v1a", "fa_tc_int8_pt", "fa", "fa_mfma", "unfused"):
            c2 = v in ("fa", "fa_mfma")
            Bs = B if not c2 else 8
            Hs = H if not c2 else 8
            Ns = N if not c2 else 1024
            # the first side measurement also absorbs the clock ramp of a fresh process
            steps_v, warm_v = (max(3, a.steps // 2), 10 if v == "fa_tc_v1a" else 2) if v != "unfused" else (3, 1)
            rv = run_variant(v, Bs, Hs, Ns, d, steps_v, warm_v, dev, rank, world)
            sib[v] = {"config": f"B{Bs} H{Hs} N{Ns} d{d}", "ms_per_step": round(rv["ms_per_step"], 4),
                      "tflops": round(flops(Bs, Hs, Ns, d) * world / (rv["ms_per_step"] * 1e-3) / 1e12, 3),
                      "main_kernel_ms": round(rv["main_kernel_ms"], 4),
                      "prepass_ms": round(rv["prepass_ms"], 4),
                      "roofline_frac": round(flops(Bs, Hs, Ns, d) / (rv["main_kernel_ms"] * 1e-3) / 1e12 /
                                             PEAKS[v], 4),
                      "peak": f"{PEAKS[v]} TFLOP/s {PEAK_KIND[v]}"}
            del rv
        side["siblings"] = sib
    if not a.no_refconfig and not dry and world == 1:
        side["reference_config"] = reference_config(a.variant, dev, rank, world)
    if not a.no_siblings and not dry and world == 1:
        side["quantize_int8"] = time_quantize_int8(B, H, N, d, dev)

    sampler = None if dry else SysfsSampler(device_state(dev).get("hwmon"))
    r = run_variant(a.variant, B, H, N, d, a.steps, a.warmup, dev, rank, world, dry_run=dry, sampler=sampler)
    total_flops = flops(B, H, N, d) * world
    value = total_flops / r["elapsed_s"] * a.steps / 1e12
    peak = PEAKS.get(a.variant, INT8_PEAK_TOPS)
    achieved = flops(B, H, N, d) / (r["main_kernel_ms"] * 1e-3) / 1e12 if r["main_kernel_ms"] > 0 else 0.0
    traffic, traffic_src = pmc_traffic(a.variant, B, H, N, d)
    busy, busy_src = pmc_sq(a.variant, B, H, N, d)
    hbm_alg = 16.0 * B * N * H * d  # fp32 Q, K, V read once + O written once (per call)
    res = {
        "metric": "attention-fwd TFLOPS + ms/call, B16 H16 N4096 d64 (fp16 & int8)",
        "value": None if dry else round(value, 3),
        "unit": "TFLOPS",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(r["ms_per_step"], 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8" if a.variant in ("fa_tc_int8_b", "fa_tc_int8_pt") else ("fp16" if a.variant == "fa_tc_v1a" else "fp32"),
        "data": ("dry run: launcher plumbing on CPU/gloo, tensor copy as the step (no kernel)" if dry else
                 "synthetic N(0, 0.5^2) fp32 Q/K/V, torch.Generator seed 1234+rank, resident in HBM"),
        "config": {"workload": f"{a.variant} attention forward (BASELINE config {'5' if world > 1 else '4'})",
                   "variant": a.variant, "B_per_gpu": B, "H": H, "N": N, "d": d, "d_model": H * d,
                   "global_batch": B * world,
                   "parallelism": f"batch-shard x{world} (no collective in the timed step; all-gather reported "
                                  f"separately)"},
    }
    if a.variant == "fa_tc_int8_b":
        # BASELINE config 4 reads "per-tensor Q/K/V quant"; the reference kernel quantises per 32-row
        # block, which is the headline; the per-tensor mode is its own variant, summarised
        # below as int8_per_tensor
        res["config"]["quantisation"] = ("per-32-row-block Q/K/V scales, per 32x32-tile P scale (the reference's "
                                         "fa_tc_int8_b numerics)")
    if dry:
        res["dry_run"] = True
    else:
        kname = f"qmha_fa_{'int8' if a.variant == 'fa_tc_int8_b' else a.variant}"
        res["roofline"] = {"bound": "mfma", "kernel": kname,
                           "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                           "frac": round(achieved / peak, 4), "traffic": traffic,
                           "traffic_source": traffic_src,
                           "algorithmic_flops_per_launch": flops(B, H, N, d),
                           "main_kernel_ms": round(r["main_kernel_ms"], 4),
                           "prepass_ms": round(r["prepass_ms"], 4),
                           "hbm_algorithmic_bytes_per_call": hbm_alg,
                           "hbm_GBs_per_call": round(hbm_alg / (r["ms_per_step"] * 1e-3) / 1e9, 1),
                           "mfma_busy_pct": busy, "mfma_busy_source": busy_src}
    if not dry:
        # reproducibility across boxes (round-5 VERDICT item 2): the clock this box holds under the kernel's
        # mix, measured right after the headline, its power cap, and the identity of the code that ran
        probe = clock_probe(dev)
        dstate = device_state(dev)
        ids = isa_ids(a.variant, d)
        res["device"] = dstate
        res["sysfs_during_timed_calls"] = sampler.summary() if sampler else None
        res["clock_probe"] = probe
        res["power_cap_w"] = dstate.get("power_cap_w")
        res["isa_sha16"] = ids.get("main", {}).get("isa_sha16")
        res["isa"] = ids
        ghz = (probe or {}).get("clock_ghz")
        res["clock_ghz"] = ghz
        if ghz and r["main_kernel_ms"] > 0:
            # wave-tiles (32 query rows x 32 keys) per SIMD of one launch
            tiles = B * H * (N // 32) ** 2 / (dstate["cus"] * 4)
            res["cycles_per_tile"] = round(r["main_kernel_ms"] * 1e-3 * ghz * 1e9 / tiles, 1)
            res["roofline"]["cycles_per_tile"] = res["cycles_per_tile"]
            res["roofline"]["tiles_per_simd"] = tiles
            # clock-free form: the tile's time in units of the probe's own unit time on the same box (the
            # ratio of two wall times; DESIGN.md 7.1: constant to +-0.3 % over five boxes)
            res["probe_units_per_tile"] = round(r["main_kernel_ms"] * 1e6 / tiles / probe["ns_per_unit_per_simd"], 4)
    if dist.is_initialized():
        ag_ms = time_allgather(r["O"], max(3, a.steps // 2), dev, world)
        sg_ms = time_solve_gather(a.variant, r["inputs"], H, d, max(3, a.steps // 2), dev, world,
                                  a.gather_chunks, dry_run=dry)
        res["allgather"] = {
            "what": f"allgather_ms: RCCL all_gather_into_tensor of every rank's [{B}, {N}, {H * d}] fp32 output "
                    f"shard into the global [{B * world}, {N}, {H * d}] on every rank, alone; step_with_allgather_ms: "
                    f"compute + copy-free gather (kernels write into their slab of the result, per-chunk "
                    f"point-to-point exchange with every peer over RCCL, overlapped with the next chunk)",
            "allgather_ms": round(ag_ms, 4),
            "step_with_allgather_ms": round(sg_ms, 4),
            "chunks": a.gather_chunks,
            "value_with_allgather": None if dry else round(total_flops / (sg_ms * 1e-3) / 1e12, 3),
        }
    del r
    res.update(side)
    pt = side.get("siblings", {}).get("fa_tc_int8_pt")
    if pt and a.variant == "fa_tc_int8_b":
        res["int8_per_tensor"] = {
            "variant": "fa_tc_int8_pt", "config": pt["config"],
            "quantisation": "one scale per (sequence, head) slice of Q/K/V, static P scale 1/127 (DESIGN.md 3.1)",
            "value": pt["tflops"], "unit": "TFLOPS", "ms_per_step": pt["ms_per_step"],
            "main_kernel_ms": pt["main_kernel_ms"], "prepass_ms": pt["prepass_ms"],
            "roofline_frac": pt["roofline_frac"]}
        tr, tr_src = pmc_traffic("fa_tc_int8_pt", B, H, N, d)
        busy_pt, busy_pt_src = pmc_sq("fa_tc_int8_pt", B, H, N, d)
        res["int8_per_tensor"].update({"traffic": tr, "traffic_source": tr_src, "mfma_busy_pct": busy_pt,
                                       "mfma_busy_source": busy_pt_src})
    if not a.no_siblings and not dry and world == 1:
        # the same call on the reference's profiling input distribution U[0, 1) (a side line; the headline
        # above is N(0, 0.5^2))
        ru = run_variant(a.variant, B, H, N, d, max(10, a.steps // 2), 10, dev, rank, world, uniform=True)
        res["uniform_inputs"] = {"data": "U[0,1) fp32 Q/K/V (reference inputs/data.cu:16-22 distribution)",
                                 "ms_per_step": round(ru["ms_per_step"], 4),
                                 "tflops": round(flops(B, H, N, d) / (ru["ms_per_step"] * 1e-3) / 1e12, 3),
                                 "main_kernel_ms": round(ru["main_kernel_ms"], 4)}
        del ru
        res["torch_ext"] = time_torch_ext(B, H, N, d, dev)
    if rank == 0 and world == 1 and not a.no_siblings and not a.no_solve_calls and not dry:
        ms = time_solve_calls(a.variant, B, H, N, d, dev)
        res["solve_calls"] = {"pattern": f"{B} blocking solve() calls, one per sequence (reference usage)",
                              "ms_per_step": round(ms, 4), "tflops": round(flops(B, H, N, d) / (ms * 1e-3) / 1e12, 3)}
    if rank == 0 and world == 1 and not a.no_cpu_baseline and not dry:
        res["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def time_quantize_int8(B, H, N, d, dev, steps=20):
    """The standalone int8 quantisation op (qmha_quantize_int8: the reference's
    fp32_to_int8sram, fa_tc_int8_b.cu:33-152, over whole tensors) on one C4-shaped fp32 tensor,
    row layout and V^T-operand layout.  HBM-bound: algorithmic bytes = fp32 in + int8 out + one
    fp32 scale per 32-row group; roofline against the ~8 TB/s HBM3E peak."""
    lib = _lib.load()
    g = torch.Generator(device=dev).manual_seed(7)
    X = torch.randn(B, N, H * d, device=dev, generator=g) * 0.5
    Xi = torch.empty(B * H * N * d, dtype=torch.int8, device=dev)
    sc = torch.empty(B * H * (N // 32), dtype=torch.float32, device=dev)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    out = {}
    for layout, name in ((0, "rows"), (1, "vt_operand")):
        def step():
            _lib.check(lib.qmha_quantize_int8(X.data_ptr(), B, N, H * d, H, Xi.data_ptr(), sc.data_ptr(), layout, sptr),
                       "quantize_int8")
        for _ in range(3):
            step()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(steps):
            step()
        s1.record()
        s1.synchronize()
        ms = s0.elapsed_time(s1) / steps
        nbytes = X.numel() * 4 + Xi.numel() + sc.numel() * 4
        out[name] = {"ms": round(ms, 4), "GB_s": round(nbytes / (ms * 1e-3) / 1e9, 1),
                     "roofline": {"bound": "hbm", "achieved": round(nbytes / (ms * 1e-3) / 1e9, 1),
                                  "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}}
    out["config"] = f"one [{B}, {N}, {H * d}] fp32 tensor, {H} heads of d={d} (a C4 operand)"
    out["algorithmic_bytes"] = X.numel() * 4 + Xi.numel() + sc.numel() * 4
    return out


def time_torch_ext(B, H, N, d, dev, steps=10):
    """The reference's Python entry point (extensions/torch/torch_ext.cpp:11-58): the compiled
    pybind `torch_ext.flash_solve(Q, K, V, d_model, num_heads, kernel)` -- one [N, d_model]
    sequence per call, blocking, as the reference binds it -- B calls per step at the C4 shape,
    beside the batched C-ABI call of the headline line (the binding's overhead)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "quantizedmha_amd", "lib"))
    try:
        import torch_ext  # the compiled pybind module (quantizedmha_amd/csrc/torch_ext.cpp)
    finally:
        sys.path.pop(0)
    g = torch.Generator(device=dev).manual_seed(11)
    Q, K, V = (torch.randn(B, N, H * d, device=dev, generator=g) * 0.5 for _ in range(3))

    def step():
        for b in range(B):
            torch_ext.flash_solve(Q[b], K[b], V[b], H * d, H, "fa_tc_int8_b")

    step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) * 1e3 / steps
    return {"pattern": f"{B} torch_ext.flash_solve calls (one [N, d_model] sequence each), kernel fa_tc_int8_b",
            "module": getattr(torch_ext, "__file__", "?"), "ms_per_step": round(ms, 4),
            "tflops": round(flops(B, H, N, d) / (ms * 1e-3) / 1e12, 3)}


def reference_config(variant, dev, rank, world):
    """The reference's own compiled configuration (include/config.h:22-28: N=8192, d_model=1024,
    h=32, so d=32) -- the shape of its published per-head times (README.md:19: 7.70 ms per head
    for fa_tc_int8_b on an L4).  One sequence, all 32 heads in one call; per-head ms beside it."""
    B, H, N, d = 1, 32, 8192, 32
    # 20 warm-up calls (3 before r03p): the clock ramps over a fresh burst's first ~20 calls
    # (tools/ramp.py -> profiles/r02/clock_ramp.txt)
    rv = run_variant(variant, B, H, N, d, 20, 20, dev, rank, world)
    pub = {"fa_tc_int8_b": 7.70}.get(variant)
    return {"config": f"B{B} H{H} N{N} d{d} (include/config.h)",
            "ms_per_call": round(rv["ms_per_step"], 4),
            "ms_per_head": round(rv["ms_per_step"] / H, 5),
            "main_kernel_ms": round(rv["main_kernel_ms"], 4),
            "tflops": round(flops(B, H, N, d) / (rv["ms_per_step"] * 1e-3) / 1e12, 3),
            "reference_ms_per_head_L4": pub}


if __name__ == "__main__":
    main()
