"""ctypes wrapper around oracle/liboracle.so and oracle/_ref/libref_verify.so.

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the quantizedmha_amd product package.
Each wrapper names the reference routine it restates (see qmha_oracle.h).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None

_f32p = ctypes.POINTER(ctypes.c_float)


def _p(a: np.ndarray, ctype=ctypes.c_float):
    return a.ctypes.data_as(ctypes.POINTER(ctype))


def build(ref: bool = False) -> None:
    """Compile liboracle.so (and, if /root/reference exists, oracle/_ref)."""
    targets = ["oracle"]
    if ref and os.path.isdir(os.environ.get("QMHA_REFERENCE", "/root/reference")):
        targets.append("ref")
    subprocess.run(["make", "-s", "-C", HERE] + targets, check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        i, f, sz, l = ctypes.c_int, ctypes.c_float, ctypes.c_size_t, ctypes.c_long
        for name in ("oracle_cpu_attention", "oracle_fa_int8", "oracle_fa_fp16", "oracle_fa_fp32", "oracle_fa_int8_pt",
                     "oracle_fa_fp16_lazy"):
            fn = getattr(L, name)
            fn.argtypes = [_f32p, _f32p, _f32p, _f32p, i, i, i, i, i]
            fn.restype = None
        L.oracle_cpu_reference_rope.argtypes = [_f32p, _f32p, _f32p, _f32p, i, i, i]
        L.oracle_cpu_reference_rope.restype = None
        L.oracle_verify_results.argtypes = [_f32p, _f32p, sz, f, f]
        L.oracle_verify_results.restype = l
        L.oracle_quantize_heads.argtypes = [_f32p, i, i, i, i, ctypes.POINTER(ctypes.c_int8), _f32p]
        L.oracle_quantize_heads.restype = None
        L.oracle_quantize_heads_pt.argtypes = [_f32p, i, i, i, i, ctypes.POINTER(ctypes.c_int8), _f32p]
        L.oracle_quantize_heads_pt.restype = None
        L.oracle_qk_int32.argtypes = [ctypes.POINTER(ctypes.c_int8), ctypes.POINTER(ctypes.c_int8), i, i,
                                      ctypes.POINTER(ctypes.c_int32)]
        L.oracle_qk_int32.restype = None
        L.oracle_f32_to_f16.argtypes = [f]
        L.oracle_f32_to_f16.restype = ctypes.c_uint16
        _LIB = L
    return _LIB


def ref_lib():
    """The reference's own utils/verify.cu (compiled into oracle/_ref)."""
    global _REF
    if _REF is None:
        path = os.path.join(HERE, "_ref", "libref_verify.so")
        if not os.path.exists(path):
            build(ref=True)
        if not os.path.exists(path):
            return None
        L = ctypes.CDLL(path)
        i = ctypes.c_int
        L.ref_cpu_reference.argtypes = [_f32p, _f32p, _f32p, _f32p, i, i, i]
        L.ref_cpu_reference.restype = None
        L.ref_verify_results.argtypes = [_f32p, _f32p, ctypes.c_size_t, ctypes.c_float, ctypes.c_float]
        L.ref_verify_results.restype = i
        _REF = L
    return _REF


def _c(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _shape(Q, d_model):
    Q = _c(Q)
    if Q.ndim == 2:
        B = 1
        N = Q.shape[0]
    else:
        B, N = Q.shape[0], Q.shape[1]
    assert Q.shape[-1] == d_model
    return B, N


def _run4(fn, Q, K, V, d_model, h, nthreads):
    Q, K, V = _c(Q), _c(K), _c(V)
    B, N = _shape(Q, d_model)
    out = np.zeros_like(Q)
    fn(_p(Q), _p(K), _p(V), _p(out), B, N, d_model, h, nthreads)
    return out


def cpu_attention(Q, K, V, d_model, h, nthreads=0):
    """tests/generate_golden.cpp:53-92 cpu_mha (no RoPE)."""
    return _run4(lib().oracle_cpu_attention, Q, K, V, d_model, h, nthreads)


def fa_int8(Q, K, V, d_model, h, nthreads=0):
    """mha_kernels/fa_tc_int8_b.cu intended algorithm."""
    return _run4(lib().oracle_fa_int8, Q, K, V, d_model, h, nthreads)


def fa_int8_pt(Q, K, V, d_model, h, nthreads=0):
    """Per-tensor int8 mode (fa_tc_int8_pt; not a reference kernel: BASELINE.json's "per-tensor
    Q/K/V quant", SURVEY 0.2's optional flag): per-head-slice scales, static P scale 1/127, lazy softmax
    base, stated in base 2 with the kernel's 22-bit score constant (qmha_oracle.c)."""
    return _run4(lib().oracle_fa_int8_pt, Q, K, V, d_model, h, nthreads)


def fa_fp16(Q, K, V, d_model, h, nthreads=0):
    """mha_kernels/fa_tc_v1a.cu."""
    return _run4(lib().oracle_fa_fp16, Q, K, V, d_model, h, nthreads)


def fa_fp16_lazy(Q, K, V, d_model, h, nthreads=0):
    """The fp16 GPU kernel's own contract (r06): fa_tc_v1a in base 2 with a lazy softmax base;
    the tests pin the kernel to it tightly and to fa_fp16 (the reference) within the fp16 bound."""
    return _run4(lib().oracle_fa_fp16_lazy, Q, K, V, d_model, h, nthreads)


def fa_fp32(Q, K, V, d_model, h, nthreads=0):
    """mha_kernels/fa.cu."""
    return _run4(lib().oracle_fa_fp32, Q, K, V, d_model, h, nthreads)


ORACLE_BY_VARIANT = {"fa_tc_int8_b": fa_int8, "fa_tc_v1a": fa_fp16, "fa": fa_fp32, "unfused": cpu_attention,
                     "fa_mfma": fa_fp32, "fa_tc_int8_pt": fa_int8_pt}


def cpu_reference_rope(Q, K, V, d_model, h):
    """utils/verify.cu:25-104 restated (single batch element, single thread)."""
    Q, K, V = _c(Q), _c(K), _c(V)
    N = Q.shape[0]
    out = np.zeros_like(Q)
    lib().oracle_cpu_reference_rope(_p(Q), _p(K), _p(V), _p(out), N, d_model, h)
    return out


def ref_cpu_reference(Q, K, V, d_model, h):
    """The reference's own cpu_reference, compiled from /root/reference."""
    L = ref_lib()
    if L is None:
        raise RuntimeError("oracle/_ref/libref_verify.so is not built")
    Q, K, V = _c(Q), _c(K), _c(V)
    N = Q.shape[0]
    out = np.zeros_like(Q)
    L.ref_cpu_reference(_p(Q), _p(K), _p(V), _p(out), N, d_model, h)
    return out


def verify_results(got, ref, eps=1e-3, rel=1e-3) -> int:
    """utils/verify.cu:153-172; returns -1 on success else the first bad index."""
    got, ref = _c(got).ravel(), _c(ref).ravel()
    return int(lib().oracle_verify_results(_p(got), _p(ref), got.size, eps, rel))


def quantize_heads(X, d_model, h):
    """Per-32-row-group int8 quantisation (fa_tc_int8_b.cu:33-152) of every head.

    Returns (Xi[B][h][N][d] int8, scales[B][h][N/32] fp32)."""
    X = _c(X)
    B, N = _shape(X, d_model)
    d = d_model // h
    Xi = np.zeros((B, h, N, d), dtype=np.int8)
    sc = np.zeros((B, h, N // 32), dtype=np.float32)
    lib().oracle_quantize_heads(_p(X), B, N, d_model, h, _p(Xi, ctypes.c_int8), _p(sc))
    return Xi, sc


def quantize_heads_pt(X, d_model, h):
    """Per-head-slice int8 quantisation (fa_tc_int8_pt): (Xi[B][h][N][d] int8, scales[B][h] fp32)."""
    X = _c(X)
    B, N = _shape(X, d_model)
    d = d_model // h
    Xi = np.zeros((B, h, N, d), dtype=np.int8)
    sc = np.zeros((B, h), dtype=np.float32)
    lib().oracle_quantize_heads_pt(_p(X), B, N, d_model, h, _p(Xi, ctypes.c_int8), _p(sc))
    return Xi, sc


def qk_int32(Qi_head, Ki_head):
    Qi_head = np.ascontiguousarray(Qi_head, dtype=np.int8)
    Ki_head = np.ascontiguousarray(Ki_head, dtype=np.int8)
    N, d = Qi_head.shape
    S = np.zeros((N, N), dtype=np.int32)
    lib().oracle_qk_int32(_p(Qi_head, ctypes.c_int8), _p(Ki_head, ctypes.c_int8), N, d, _p(S, ctypes.c_int32))
    return S


def f32_to_f16_bits(x: float) -> int:
    return int(lib().oracle_f32_to_f16(float(x)))


def fp32_reference_attention(Q, K, V, d_model, h):
    """float64 numpy attention (independent of the restatements) for tolerance checks."""
    Q = np.asarray(Q, dtype=np.float64)
    K = np.asarray(K, dtype=np.float64)
    V = np.asarray(V, dtype=np.float64)
    squeeze = Q.ndim == 2
    if squeeze:
        Q, K, V = Q[None], K[None], V[None]
    B, N, _ = Q.shape
    d = d_model // h
    q = Q.reshape(B, N, h, d).transpose(0, 2, 1, 3)
    k = K.reshape(B, N, h, d).transpose(0, 2, 1, 3)
    v = V.reshape(B, N, h, d).transpose(0, 2, 1, 3)
    s = q @ k.transpose(0, 1, 3, 2) / np.sqrt(d)
    s -= s.max(-1, keepdims=True)
    p = np.exp(s)
    p /= p.sum(-1, keepdims=True)
    o = (p @ v).transpose(0, 2, 1, 3).reshape(B, N, d_model)
    return o[0] if squeeze else o
