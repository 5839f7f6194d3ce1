#!/usr/bin/env python3
"""Numerical pre-checks (round 4) of two int8 restructurings, against the per-block contract.

Self-contained numpy restatement of the per-block int8 algorithm (the same steps as
oracle/qmha_oracle.c fa_int8_item, re-derived here so this tool touches nothing under oracle/),
vectorised over the 32-row query groups of one head, in three forms:

  seq     the contract: one online-softmax sweep over all KV tiles, m0 = 0 (fa_tc_int8_b.cu:402)
  split   the KV sweep cut into S chunks, each chunk started at m = 0, l = 0, O = 0, combined at
          the end by the usual max-rescale (a split-KV / flash-decoding occupancy path); with
          --exact-m each chunk starts from the running max the sequential sweep has at its first
          tile (what a split path would have to compute first to keep the contract)
  f16acc  P@V accumulated across tiles in the MFMA accumulator: the per-(row, tile) fold scale
          sP * sV * 2^(m - anchor) moved into the P operand, P' = f16(Pi * f16(scale)), O in fp32
          (anchored, re-anchored past 8 log2 units, per-head power-of-two
          normaliser on sV so P' stays in f16's normal range)

Prints max |form - seq| and the fraction of elements above 5e-5, the GPU parity criteria
(tests/test_gpu_parity.py int8_tol: 1e-4 at N >= 2048, 5e-4 below; at most 0.2 % above 5e-5).
    python tools/numerics_r04.py            # C4-like, reference-config-like and peaked inputs
"""
import argparse

import numpy as np

f32 = np.float32


def quant(X):
    """fa_tc_int8_b.cu:33-152 per 32-row group: s = max(absmax/127, 1e-8), rint(x * (1/s)) clamped."""
    am = np.abs(X).reshape(X.shape[0], -1).max(1)
    s = np.maximum(am / f32(127), f32(1e-8)).astype(f32)
    inv = (f32(1) / s).astype(f32)
    return np.clip(np.rint(X * inv[:, None, None]), -128, 127).astype(np.int32), s


def tile_step(acc, sQ, sKt, isd, m):
    s = ((acc.astype(f32) * sQ[:, None, None]).astype(f32) * sKt).astype(f32) * isd
    m_new = np.maximum(m, s.max(2))
    p = np.exp(s - m_new[:, :, None]).astype(f32)
    pm = p.reshape(p.shape[0], -1).max(1)
    sP = np.maximum(pm / f32(127), f32(1e-8)).astype(f32)
    Pi = np.clip(np.rint(p * (f32(1) / sP)[:, None, None]), -128, 127).astype(np.int32)
    return m_new, p.sum(2, dtype=f32), sP, Pi


def head(Q, K, V, form, nsplit=1, exact_m=False, bound_log2=8.0):
    N, d = Q.shape
    G = N // 32
    Qi, sQ = quant(Q.reshape(G, 32, d))
    Ki, sK = quant(K.reshape(G, 32, d))
    Vi, sV = quant(V.reshape(G, 32, d))
    isd = f32(1 / np.sqrt(d))
    S = [Qi @ Ki[t].T for t in range(G)]  # int32 scores per tile [G, 32, 32]
    if form == "f16acc":
        O = np.zeros((G, 32, d), f32)
        l = np.zeros((G, 32), f32)
        m = np.zeros((G, 32), f32)
        anchor = np.zeros((G, 32), f32)
        norm = f32(2.0 ** np.ceil(np.log2(sV.max())))
        for t in range(G):
            m_new, rs, sP, Pi = tile_step(S[t], sQ, sK[t], isd, m)
            re = (m_new - anchor) > f32(bound_log2 * np.log(2))
            if re.any():
                f = np.where(re, np.exp(anchor - m_new), f32(1)).astype(f32)
                O *= f[:, :, None]
                l *= f
                anchor = np.where(re, m_new, anchor)
            e = np.exp(m_new - anchor).astype(f32)
            l = l + rs * e
            c = (sP[:, None] * sV[t] * e / norm).astype(np.float16).astype(f32)
            Pp = (Pi.astype(f32) * c[:, :, None]).astype(np.float16).astype(f32)
            O = O + (Pp @ Vi[t].astype(f32)).astype(f32)
            m = m_new
        un = np.exp(anchor - m).astype(f32)
        L = l * un
        return np.where(L[:, :, None] > 1e-20, O * norm * un[:, :, None] / L[:, :, None], 0).reshape(N, d)
    # seq / split: chunk k covers tiles [b_k, b_{k+1})
    bounds = [G * k // nsplit for k in range(nsplit + 1)]
    m_seq = np.zeros((G, 32), f32)  # running max of the sequential sweep (for exact_m)
    starts = {}
    for t in range(G):
        if t in bounds:
            starts[t] = m_seq.copy()
        m_seq = np.maximum(m_seq, (((S[t].astype(f32) * sQ[:, None, None]).astype(f32) * sK[t]).astype(f32) * isd).max(2))
    Of = np.zeros((G, 32, d), np.float64)
    lf = np.zeros((G, 32), np.float64)
    mf = np.full((G, 32), -np.inf)
    for k in range(nsplit):
        O = np.zeros((G, 32, d), f32)
        l = np.zeros((G, 32), f32)
        m = starts[bounds[k]].copy() if exact_m else np.zeros((G, 32), f32)
        for t in range(bounds[k], bounds[k + 1]):
            m_new, rs, sP, Pi = tile_step(S[t], sQ, sK[t], isd, m)
            alpha = np.exp(m - m_new).astype(f32)
            l = alpha * l + rs
            O = O * alpha[:, :, None] + (Pi @ Vi[t]).astype(f32) * sP[:, None, None] * sV[t]
            m = m_new
        mn = np.maximum(mf, m)
        a, b = np.exp(mf - mn), np.exp(m - mn)
        Of = Of * a[:, :, None] + O * b[:, :, None]
        lf = lf * a + l * b
        mf = mn
    return np.where(lf[:, :, None] > 1e-20, Of / lf[:, :, None], 0).astype(f32).reshape(N, d)


def compare(name, Q, K, V, h):
    d = Q.shape[1] // h
    seq, forms = [], {}
    cases = [("split2", dict(form="split", nsplit=2)), ("split3", dict(form="split", nsplit=3)),
             ("split2-exact-m", dict(form="split", nsplit=2, exact_m=True)), ("f16acc", dict(form="f16acc"))]
    for k in range(h):
        sl = slice(k * d, (k + 1) * d)
        ref = head(Q[:, sl], K[:, sl], V[:, sl], "seq")
        for cname, kw in cases:
            forms.setdefault(cname, []).append(np.abs(head(Q[:, sl], K[:, sl], V[:, sl], **kw) - ref))
    for cname, errs in forms.items():
        e = np.concatenate(errs)
        print(f"{name:>10s} {cname:>15s}  max|form - seq| {e.max():.3g}  frac > 5e-5 {(e > 5e-5).mean():.4f}", flush=True)


def main():
    argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter).parse_args()
    rng = np.random.default_rng(1)
    N, h, d = 4096, 2, 64  # BASELINE C4 data (tests/test_gpu_parity.py: Q, K ~ 0.5 N(0,1), V ~ U[0,1))
    compare("C4", (rng.standard_normal((N, h * d)) * 0.5).astype(f32), (rng.standard_normal((N, h * d)) * 0.5).astype(f32),
            rng.random((N, h * d)).astype(f32), h)
    N, h, d = 8192, 2, 32  # the reference's own shape and data (include/config.h:22-28, U[0,1))
    compare("refconfig", *(rng.random((N, h * d)).astype(f32) for _ in range(3)), h)
    N, dm, h = 512, 128, 2  # tests/test_gpu_parity.py test_growing_scores_reanchor inputs
    r7 = np.random.default_rng(7)
    Q = (r7.standard_normal((N, dm)) * 0.2 + 1.0).astype(f32)
    ramp = np.linspace(0.0, 4.0, N, dtype=f32)[:, None]
    K = ((r7.standard_normal((N, dm)) * 0.2 + 1.0) * ramp).astype(f32)
    compare("growing", Q, K, r7.standard_normal((N, dm)).astype(f32), h)
    N, h, d = 1024, 2, 64  # peaked rows: wide scores
    compare("peaked", *((rng.standard_normal((N, h * d)) * 1.5).astype(f32) for _ in range(3)), h)


if __name__ == "__main__":
    main()
