#!/usr/bin/env python3
"""Regenerate the committed golden fixtures under tests/golden/ from the REFERENCE.

Run in the build container (needs /root/reference):  python tests/golden/make_golden.py

1. Builds oracle/_ref/generate_golden from /root/reference/tests/generate_golden.cpp
   (unmodified) and runs it in a scratch directory.  It writes tests/golden/<case>/
   {Q,K,V,O,S,P}.f32.bin + meta.json (generate_golden.cpp:148-161).  We keep:
     small, unaligned, quant_small  -- all files (tiny)
     medium (N=128,d_model=512,h=8) -- heads 0-3 sliced out  (d = 64)
     large  (N=256,d_model=1024,h=16) -- heads 0-1 sliced out (d = 64)
     huge_1024 (N=1024,d_model=128,h=8) -- head 0 sliced out (d = 16)
   A head's output depends only on its own column slice, so a slice of a golden
   case is itself a golden case (meta.json records the source).
2. Builds oracle/_ref/ref_inputs (restating inputs/data.cu:9-30's mt19937(42)
   U[0,1) generator) and oracle/_ref/libref_verify.so (the reference's own
   utils/verify.cu) and writes the driver's caches in the reference's formats:
     c1_verify/input_random_N128_d128.bin  (data.cu:54-108: int N, int d_model, Q, K, V)
     c1_verify/ref_N128_d128.bin           (verify.cu:106-124: int N, int d_model, out)
   where out = cpu_reference (RoPE) for config 1 (B1 H2 N128 d64), and the same
   for the all-ones correctness-check input (c1_ones/).
"""
import ctypes
import json
import os
import shutil
import struct
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
SLICES = {"medium": 4, "large": 2, "huge_1024": 1}
FULL = ["small", "unaligned", "quant_small"]


def slice_case(src, dst, heads):
    meta = json.load(open(os.path.join(src, "meta.json")))
    N, dm, h = meta["N"], meta["d_model"], meta["h"]
    d = dm // h
    cols = heads * d
    os.makedirs(dst, exist_ok=True)
    for t in ("Q", "K", "V", "O"):
        a = np.fromfile(os.path.join(src, f"{t}.f32.bin"), dtype=np.float32).reshape(N, dm)
        np.ascontiguousarray(a[:, :cols]).tofile(os.path.join(dst, f"{t}.f32.bin"))
    meta_out = {"N": N, "d_model": cols, "h": heads,
                "source": f"generate_golden.cpp case with d_model={dm}, h={h}; heads 0..{heads - 1}"}
    json.dump(meta_out, open(os.path.join(dst, "meta.json"), "w"), indent=2)


def write_inputs_cache(path, N, dm, Q, K, V):
    with open(path, "wb") as f:
        f.write(struct.pack("ii", N, dm))
        for a in (Q, K, V):
            f.write(np.ascontiguousarray(a, dtype=np.float32).tobytes())


def write_ref_cache(path, N, dm, out):
    with open(path, "wb") as f:
        f.write(struct.pack("ii", N, dm))
        f.write(np.ascontiguousarray(out, dtype=np.float32).tobytes())


def main():
    oracle.build(ref=True)
    ref_dir = os.path.join(ROOT, "oracle", "_ref")
    with tempfile.TemporaryDirectory() as tmp:
        subprocess.run([os.path.join(ref_dir, "generate_golden")], cwd=tmp, check=True,
                       stdout=subprocess.DEVNULL)
        src = os.path.join(tmp, "tests", "golden")
        for case in FULL:
            dst = os.path.join(GOLD, case)
            shutil.rmtree(dst, ignore_errors=True)
            shutil.copytree(os.path.join(src, case), dst)
        for case, heads in SLICES.items():
            dst = os.path.join(GOLD, case)
            shutil.rmtree(dst, ignore_errors=True)
            slice_case(os.path.join(src, case), dst, heads)

        # config-1 verify-path caches in the reference's own formats
        N, dm, h = 128, 128, 2
        for name, extra in (("c1_verify", []), ("c1_ones", ["ones"])):
            dst = os.path.join(GOLD, name)
            os.makedirs(dst, exist_ok=True)
            raw = os.path.join(tmp, f"{name}.bin")
            subprocess.run([os.path.join(ref_dir, "ref_inputs"), str(N), str(dm), raw] + extra, check=True)
            buf = open(raw, "rb").read()
            n = N * dm
            arr = np.frombuffer(buf[8:], dtype=np.float32)
            Q, K, V = (arr[i * n:(i + 1) * n].reshape(N, dm) for i in range(3))
            out = oracle.ref_cpu_reference(Q, K, V, dm, h)
            kind = "input_random" if not extra else "input_ones"
            write_inputs_cache(os.path.join(dst, f"{kind}_N{N}_d{dm}.bin"), N, dm, Q, K, V)
            write_ref_cache(os.path.join(dst, f"ref_N{N}_d{dm}.bin"), N, dm, out)
            json.dump({"N": N, "d_model": dm, "h": h,
                       "source": "inputs/data.cu:9-30 generator + utils/verify.cu cpu_reference (RoPE), "
                                 "compiled from /root/reference"},
                      open(os.path.join(dst, "meta.json"), "w"), indent=2)
    print("golden fixtures written under", GOLD)


if __name__ == "__main__":
    main()
