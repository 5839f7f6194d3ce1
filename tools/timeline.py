#!/usr/bin/env python3
"""Per-workgroup timeline of the int8 pipelined main kernel (QMHA_TIMELINE profiling build only).

    bash tools/alt_build.sh tl -DQMHA_TIMELINE
    QMHA_LIB_PATH=quantizedmha_amd/alt_lib/tl/libqmha.so python tools/timeline.py <variant> B H N d

Runs 25 calls, then reads each workgroup's start / end wall clock (s_memrealtime, 100 MHz) and its
hardware slot of the LAST launch, and prints: the kernel span, the workgroup-duration spread, how
many workgroups start within the first microseconds (the first round), and how the number of
resident workgroups falls off at the end (the ragged end) -- i.e. where the kernel's time goes
beyond its steady state.
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizedmha_amd import _lib, torch_ext  # noqa: E402

TICK_NS = 10.0  # s_memrealtime: 100 MHz


def main():
    variant = sys.argv[1]
    B, H, N, d = (int(x) for x in sys.argv[2:6])
    lib = _lib.load()
    fn = lib.qmha_debug_timeline
    fn.argtypes = [ctypes.c_void_p]
    fn.restype = ctypes.c_int
    g = torch.Generator(device="cuda").manual_seed(1234)
    Q, K, V = (torch.randn(B, N, H * d, device="cuda", generator=g) * 0.5 for _ in range(3))
    for _ in range(25):
        out = torch_ext.flash_solve(Q, K, V, H * d, H, kernel=variant)
    torch.cuda.synchronize()
    buf = np.zeros((4, 1 << 17), np.uint64)
    assert fn(buf.ctypes.data) == 0
    nwg = B * H * ((N // 32 + 3) // 4)
    t0, t1 = buf[0, :nwg].astype(np.int64), buf[1, :nwg].astype(np.int64)
    assert (t1 > 0).all() and (t1 >= t0).all(), "timeline not recorded (not a QMHA_TIMELINE build?)"
    base = t0.min()
    s, e = (t0 - base) * TICK_NS / 1e3, (t1 - base) * TICK_NS / 1e3  # microseconds
    dur = e - s
    span = e.max()
    hw, xcc = buf[2, :nwg].astype(np.int64), buf[3, :nwg].astype(np.int64) & 0xF
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    print(f"{variant} B{B} H{H} N{N} d{d}: {nwg} workgroups, span {span:.1f} us (first start -> last end)")
    print(f"  workgroup duration: mean {dur.mean():.1f} us, min {dur.min():.1f}, p50 {np.median(dur):.1f}, "
          f"p95 {np.percentile(dur, 95):.1f}, max {dur.max():.1f}")
    r1 = s < 2.0
    first = r1.sum()
    print(f"  started within 2 us: {first} workgroups (the first round); last start at {s.max():.1f} us")
    later = ~r1 & (s < s.max() - dur.mean())  # neither the first round nor the drain
    print(f"  duration, first round: mean {dur[r1].mean():.1f} us (p05 {np.percentile(dur[r1], 5):.1f}, p95 "
          f"{np.percentile(dur[r1], 95):.1f}); steady-state starts: "
          + (f"mean {dur[later].mean():.1f} us (n={later.sum()})" if later.any() else "none"))
    grid = np.linspace(0, span, 201)
    resident = np.array([((s <= t) & (e > t)).sum() for t in grid])
    peak = resident.max()
    full = grid[resident >= 0.95 * peak]
    tail_start = full.max() if len(full) else 0.0
    print(f"  resident workgroups: peak {peak}; >= 95 % of peak until {tail_start:.1f} us; "
          f"mean occupancy over the span {resident.mean() / peak:.3f} of peak")
    print(f"  ragged end: {span - tail_start:.1f} us ({(span - tail_start) / span:.1%} of the span)")
    for x in range(8):
        m = xcc == x
        if m.any():
            print(f"  xcc {x}: {m.sum():5d} wg, mean duration {dur[m].mean():.1f} us, last end {e[m].max():.1f} us, "
                  f"CUs {len(set(zip(se[m].tolist(), cu[m].tolist())))}")
    print("  resident-count profile (every 10th of 201 points): " +
          " ".join(str(int(r)) for r in resident[::10]))


if __name__ == "__main__":
    main()
