"""Readers for the committed golden fixtures (reference formats, see tests/golden/make_golden.py)."""
import json
import os
import struct

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["small", "unaligned", "medium", "large", "huge_1024", "quant_small"]


def load_case(name):
    d = os.path.join(GOLD, name)
    m = json.load(open(os.path.join(d, "meta.json")))
    N, dm, h = m["N"], m["d_model"], m["h"]
    r = {t: np.fromfile(os.path.join(d, f"{t}.f32.bin"), dtype=np.float32).reshape(N, dm) for t in "QKVO"}
    return N, dm, h, r["Q"], r["K"], r["V"], r["O"]


def load_inputs_cache(path):
    """inputs/data.cu:54-108 format: int N, int d_model, Q, K, V."""
    b = open(path, "rb").read()
    N, dm = struct.unpack("ii", b[:8])
    a = np.frombuffer(b[8:], dtype=np.float32)
    n = N * dm
    return N, dm, [a[i * n:(i + 1) * n].reshape(N, dm).copy() for i in range(3)]


def load_ref_cache(path):
    """utils/verify.cu:106-151 format: int N, int d_model, out."""
    b = open(path, "rb").read()
    N, dm = struct.unpack("ii", b[:8])
    return N, dm, np.frombuffer(b[8:], dtype=np.float32).reshape(N, dm).copy()
