"""GPU parity tests (MI355X): every variant through the C-ABI against the CPU oracle.

Tolerances (stated per SURVEY 8c; the oracle restates the reference algorithm, the GPU
kernels deviate only in fp32 rounding order and the exp implementation):
  * int8: quantised Q/K/V bytes and scales, and int32 Q@K^T -> bit-exact
          O vs oracle fa_int8, bound by sequence length (int8_tol): an exp ulp can flip one
          P rounding, which moves a row by sP*sV*|Vi|/l, and l grows with N:
            N <= 256   every element <= 2e-3, all but 0.2 % <= 5e-5
            N <  2048  every element <= 5e-4, all but 0.2 % <= 5e-5
            N >= 2048  every element <= 1e-4, all but 0.2 % <= 5e-5 -- the
                       BASELINE C4/C5 and reference-config cases
          O vs fp32 attention golden <= 5e-3 abs (quantisation error budget)
  * fp16: O vs oracle fa_fp16 <= 2e-4, vs golden within verify.cu's 1e-3 abs/rel
  * fp32: O vs oracle fa_fp32 <= 1e-5 abs
  * unfused: O vs cpu_attention <= 1e-5 abs
The observed maximum of every case is printed in pytest's terminal summary (tests/parity_log.py).
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from tests import parity_log
from tests.golden_io import load_case

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# int8 vs oracle: the GPU's exp2 and the oracle's expf differ in the last ulp, which can move
# p/sP across a .5 rounding boundary and change one Pi by 1.  One such flip moves O by
# sP*sV*|Vi|/l (up to ~1e-3 at N=128, ~1e-5 at N=4096), so the int8 check is statistical: every
# element within int8_tol(N), and all but INT8_FLIP_FRAC of the elements within INT8_TOL_TIGHT.
INT8_TOL_TIGHT = 5e-5
INT8_FLIP_FRAC = 2e-3
TOL_ORACLE = {"fa_tc_int8_b": 2e-3, "fa_tc_v1a": 2e-4, "fa": 1e-5, "fa_mfma": 1e-5, "unfused": 1e-5,
              "fa_tc_int8_pt": 2e-3}
TOL_GOLDEN = {"fa_tc_int8_b": 5e-3, "fa_tc_v1a": 1e-3, "fa": 1e-5, "fa_mfma": 1e-5, "unfused": 1e-5,
              "fa_tc_int8_pt": 5e-3}
VARIANTS = list(TOL_ORACLE)
# fa_tc_int8_pt (the per-tensor mode, oracle fa_int8_pt) flips like fa_tc_int8_b, with int8_tol; each flip
# weighs (1/127) sV |Vi| / l with the head-slice sV (larger than a 32-row group's), so its budget of
# elements above 5e-5 is 0.5 %.  Since r06 the oracle states the kernel's base-2 contract (the 22-bit
# score constant, x rounded once): what is left to flip a Pi is the exp2 ulp and the KFOLD row factor
INT8_VARIANTS = ("fa_tc_int8_b", "fa_tc_int8_pt")
INT8_FLIP_FRAC_PT = 5e-3


def int8_tol(N):
    """Max |O_gpu - O_oracle| for fa_tc_int8_b at sequence length N (see the module docstring)."""
    if N <= 256:
        return 2e-3
    if N < 2048:
        return 5e-4
    return 1e-4


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from quantizedmha_amd import _lib
    _lib.load()  # raises if the HIP library is missing: no silent fallback
    return torch.device("cuda:0")


def oracle_for(oracle_mod, variant):
    return oracle_mod.ORACLE_BY_VARIANT[variant]


def assert_parity(variant, out, ref, scale=1.0, N=None):
    """out/ref: [..., N, d_model]; N defaults to out.shape[-2] (the sequence length)."""
    err = np.abs(np.asarray(out, np.float64) - np.asarray(ref, np.float64))
    assert np.isfinite(out).all()
    n = int(N if N is not None else np.asarray(out).shape[-2])
    tol = (int8_tol(n) if variant in INT8_VARIANTS else TOL_ORACLE[variant]) * scale
    frac = float((err > INT8_TOL_TIGHT).mean())
    parity_log.record(os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0].split("::")[-1], variant,
                      err.max(), frac, tol)
    assert err.max() <= tol, (variant, float(err.max()), tol)
    if variant in INT8_VARIANTS:
        assert frac <= (INT8_FLIP_FRAC_PT if variant == "fa_tc_int8_pt" else INT8_FLIP_FRAC), (frac, float(err.max()))


def run(variant, Q, K, V, d_model, h, dev):
    from quantizedmha_amd import torch_ext
    t = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (Q, K, V)]
    out = torch_ext.flash_solve(t[0], t[1], t[2], d_model, h, kernel=variant)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def rand_inputs(seed, B, N, d_model, dist="normal"):
    rng = np.random.default_rng(seed)
    shape = (B, N, d_model) if B > 1 else (N, d_model)
    if dist == "normal":
        return [(rng.standard_normal(shape) * 0.5).astype(np.float32) for _ in range(3)]
    return [rng.random(shape, dtype=np.float32) for _ in range(3)]


# --------------------------------------------------------------------------------------
# INT8 exact pieces
# --------------------------------------------------------------------------------------
@pytest.mark.parametrize("N,d_model,h", [(64, 64, 2), (128, 256, 4), (96, 128, 1), (256, 128, 2),
                                         (96, 192, 2), (64, 320, 2), (64, 512, 2)])  # d = 96, 160, 256
def test_int8_quantised_bytes_and_scales_bitexact(dev, oracle_mod, N, d_model, h):
    from quantizedmha_amd import torch_ext
    X = rand_inputs(1, 1, N, d_model)[0]
    X[3, 5] = 7.0  # scale outlier
    X[N - 32:] *= 1e-9  # a group near the 1e-8 scale floor
    Xi_ref, sc_ref = oracle_mod.quantize_heads(X, d_model, h)
    Xg, scg = torch_ext.quantize_int8(torch.from_numpy(X).to(dev), d_model, h, layout=0)
    assert np.array_equal(scg.cpu().numpy(), sc_ref)
    assert np.array_equal(Xg.cpu().numpy(), Xi_ref)
    # layout 1: V^T operand order [B][h][N/32][d][32] with the i8 slot permutation
    Vg, scv = torch_ext.quantize_int8(torch.from_numpy(X).to(dev), d_model, h, layout=1)
    assert np.array_equal(scv.cpu().numpy(), sc_ref)
    d = d_model // h
    kv_of_slot = [(s & 3) + 8 * ((s & 15) >> 2) + 4 * (s >> 4) for s in range(32)]
    ref_t = Xi_ref.reshape(1, h, N // 32, 32, d)[:, :, :, kv_of_slot, :].transpose(0, 1, 2, 4, 3)
    assert np.array_equal(Vg.cpu().numpy(), ref_t)


@pytest.mark.parametrize("N,d_model,h", [(64, 64, 2), (256, 128, 2), (96, 256, 2), (4096, 1024, 16)])
def test_int8_pt_quantised_bytes_and_scales_bitexact(dev, oracle_mod, N, d_model, h):
    """The per-tensor mode's quantiser (group absmax pass + one scale per head slice, the
    fa_tc_int8_pt pre-pass) through the quantisation op's layout 2: int8 rows and the [B][h]
    scales bit for bit against the oracle's per-slice fp32_to_int8sram."""
    from quantizedmha_amd import torch_ext
    X = rand_inputs(5, 2, N, d_model)[0]
    X[0, 3, 5] = 7.0  # a slice-wide outlier
    X[1, :, :d_model // h] *= 1e-9  # a head slice at the 1e-8 scale floor
    Xi_ref, sc_ref = oracle_mod.quantize_heads_pt(X, d_model, h)
    Xg, scg = torch_ext.quantize_int8(torch.from_numpy(X).to(dev), d_model, h, layout=2)
    assert np.array_equal(scg.cpu().numpy(), sc_ref)
    assert np.array_equal(Xg.cpu().numpy(), Xi_ref)


def test_int8_pt_full_config_all_heads(dev, oracle_mod):
    """The per-tensor mode at the C4 shape (B16 H16 N4096 d64): all 256 (batch, head) slices against
    oracle fa_int8_pt at the N >= 2048 bound (1e-4), outputs inside [0, 1]."""
    from quantizedmha_amd import torch_ext
    B, N, H, d = 16, 4096, 16, 64
    g = torch.Generator(device=dev).manual_seed(4)
    Q = torch.randn(B, N, H * d, device=dev, generator=g) * 0.5
    K = torch.randn(B, N, H * d, device=dev, generator=g) * 0.5
    V = torch.rand(B, N, H * d, device=dev, generator=g)
    out = torch_ext.flash_solve(Q, K, V, H * d, H, kernel="fa_tc_int8_pt")
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    assert float(out.min()) >= 0.0 and float(out.max()) <= 1.0
    got, ref = _all_slices_vs_oracle(oracle_mod.fa_int8_pt, Q, K, V, out, d)
    assert_parity("fa_tc_int8_pt", got, ref, N=N)
    for b in (0, 15):  # one sequence per call (issue-priority fairness on): bit-identical slices
        one = torch_ext.flash_solve(Q[b], K[b], V[b], H * d, H, kernel="fa_tc_int8_pt")
        torch.cuda.synchronize()
        assert torch.equal(one, out[b]), b


@pytest.mark.parametrize("B,N,H,d", [(4, 4096, 16, 64), (2, 1024, 8, 32), (2, 2048, 4, 128), (3, 96, 2, 64)])
def test_int8_pt_prepass_fallback_bit_identical(dev, B, N, H, d):
    """The per-tensor pre-pass holds each part of a head slice in registers and waits (bounded) for the
    slice's other parts; past the bound a part reduces the whole slice itself.  Forcing
    that fallback for every part (qmha_debug_set_pt_wait(0)) must give the same bytes, scales and output."""
    from quantizedmha_amd import _lib, torch_ext
    lib = _lib.load()
    g = torch.Generator(device=dev).manual_seed(21)
    Q, K, V = (torch.randn(B, N, H * d, device=dev, generator=g) * 0.5 for _ in range(3))
    V[0, 5, 3] = 9.0  # a slice-wide outlier: the scale the fallback must find too
    ref = torch_ext.flash_solve(Q, K, V, H * d, H, kernel="fa_tc_int8_pt")
    refq = torch_ext.quantize_int8(K, H * d, H, layout=2)
    torch.cuda.synchronize()
    prev = lib.qmha_debug_set_pt_wait(0)
    try:
        out = torch_ext.flash_solve(Q, K, V, H * d, H, kernel="fa_tc_int8_pt")
        q = torch_ext.quantize_int8(K, H * d, H, layout=2)
        torch.cuda.synchronize()
        lib.qmha_debug_set_pt_wait(-1)  # the two-pass form (absmax launch, then quantisation launch)
        out2 = torch_ext.flash_solve(Q, K, V, H * d, H, kernel="fa_tc_int8_pt")
        q2 = torch_ext.quantize_int8(K, H * d, H, layout=2)
        torch.cuda.synchronize()
    finally:
        lib.qmha_debug_set_pt_wait(prev)
    assert prev == 200000
    assert torch.equal(out, ref)
    assert torch.equal(q[0], refq[0]) and torch.equal(q[1], refq[1])
    assert torch.equal(out2, ref)
    assert torch.equal(q2[0], refq[0]) and torch.equal(q2[1], refq[1])


def test_int8_pt_long_slices_two_pass(dev, oracle_mod):
    """Head slices of more parts than one XCD holds at once (d = 128, N = 16384: 43 parts of 12 groups per
    K / V slice against ~32 resident pre-pass workgroups per XCD) take the two-pass pre-pass (round-4 ADVICE:
    the single read would leave every part waiting out its 2 ms bound).  Checked: the quantised bytes and
    slice scales bit for bit against the oracle, sampled rows against exact fp64 attention, and a call time
    far below what one 2 ms wait per part would cost."""
    import time
    from quantizedmha_amd import torch_ext
    N, dm, h = 16384, 256, 2
    d = dm // h
    Q, K, V = rand_inputs(77, 1, N, dm)
    K[9, 3] = 6.0  # slice-wide outlier
    Xi_ref, sc_ref = oracle_mod.quantize_heads_pt(K[None], dm, h)
    Xg, scg = torch_ext.quantize_int8(torch.from_numpy(K[None]).to(dev), dm, h, layout=2)
    assert np.array_equal(scg.cpu().numpy(), sc_ref)
    assert np.array_equal(Xg.cpu().numpy(), Xi_ref)
    t = [torch.from_numpy(x).to(dev) for x in (Q, K, V)]
    out = torch_ext.flash_solve(t[0], t[1], t[2], dm, h, kernel="fa_tc_int8_pt")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        out = torch_ext.flash_solve(t[0], t[1], t[2], dm, h, kernel="fa_tc_int8_pt")
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / 5
    out = out.cpu().numpy()
    assert np.isfinite(out).all()
    rows = np.unique(np.concatenate([np.linspace(0, N - 1, 62).astype(int), [1, N - 2]]))
    err = 0.0
    for k in range(h):
        c = slice(k * d, (k + 1) * d)
        S = Q[rows, c].astype(np.float64) @ K[:, c].astype(np.float64).T / np.sqrt(d)
        P = np.exp(S - S.max(axis=1, keepdims=True))
        ref = (P / P.sum(axis=1, keepdims=True)) @ V[:, c].astype(np.float64)
        err = max(err, float(np.abs(out[rows, c] - ref).max()))
    parity_log.record("test_int8_pt_long_slices_two_pass", "fa_tc_int8_pt (vs fp64)", err, 0.0,
                      TOL_FP64["fa_tc_int8_pt"])
    assert err <= TOL_FP64["fa_tc_int8_pt"], err
    assert ms < 20.0, ms  # ~2 ms of compute; 43 parts x 2 ms of waiting would be far above this


def test_int8_nan_inputs(dev, oracle_mod):
    """NaN in the caller's Q / K / V (the pre-passes keep IEEE semantics, round-2 ADVICE; the main
    kernel's in-register Q quantiser zeroes NaNs by an integer test on the bits): the
    reference's quantiser drops a NaN from the group absmax (fmaxf) and __float2int_rn turns it into
    0, so the int8 path's output stays finite and equals the oracle's; the quantisation op writes the
    same bytes and scales bit for bit."""
    from quantizedmha_amd import torch_ext
    N, dm, h = 256, 128, 2
    Q, K, V = rand_inputs(61, 1, N, dm)
    for X, pos in ((Q, [(3, 7), (100, 64)]), (K, [(0, 0), (37, 127)]), (V, [(200, 5), (31, 70)])):
        for r, c in pos:
            X[r, c] = np.nan
    Xg, scg = torch_ext.quantize_int8(torch.from_numpy(K).to(dev), dm, h, layout=0)
    Ki_ref, sk_ref = oracle_mod.quantize_heads(K, dm, h)
    assert np.array_equal(scg.cpu().numpy(), sk_ref) and np.isfinite(sk_ref).all()
    assert np.array_equal(Xg.cpu().numpy(), Ki_ref)
    assert Ki_ref[0, 0, 0, 0] == 0 and Ki_ref[0, 1, 37, 63] == 0  # the NaN elements
    out = run("fa_tc_int8_b", Q, K, V, dm, h, dev)
    ref = oracle_mod.fa_int8(Q, K, V, dm, h)
    assert np.isfinite(ref).all()
    assert_parity("fa_tc_int8_b", out, ref)
    # the per-tensor mode (round-3 ADVICE): slice absmax from the IEEE pre-pass, Q quantised in the
    # main kernel with its NaNs zeroed explicitly (qmha_fa_int8.hip nan_to_zero), the layout-2 bytes
    out = run("fa_tc_int8_pt", Q, K, V, dm, h, dev)
    ref = oracle_mod.fa_int8_pt(Q, K, V, dm, h)
    assert np.isfinite(ref).all()
    assert_parity("fa_tc_int8_pt", out, ref)
    Xg, scg = torch_ext.quantize_int8(torch.from_numpy(Q).to(dev), dm, h, layout=2)
    Qi_ref, sq_ref = oracle_mod.quantize_heads_pt(Q, dm, h)
    assert np.array_equal(scg.cpu().numpy(), sq_ref) and np.array_equal(Xg.cpu().numpy(), Qi_ref)


@pytest.mark.parametrize("N,d_model,h,head", [(128, 128, 2, 1), (256, 64, 2, 0), (64, 128, 1, 0), (128, 512, 4, 3),
                                              (128, 192, 2, 1), (64, 256, 1, 0)])  # d = 96, 256
def test_int8_qk_int32_bitexact(dev, oracle_mod, N, d_model, h, head):
    from quantizedmha_amd import torch_ext
    Q, K, _ = rand_inputs(2, 1, N, d_model)
    S = torch_ext.debug_qk_int32(torch.from_numpy(Q).to(dev), torch.from_numpy(K).to(dev), d_model, h, head)
    Qi, _ = oracle_mod.quantize_heads(Q, d_model, h)
    Ki, _ = oracle_mod.quantize_heads(K, d_model, h)
    S_ref = oracle_mod.qk_int32(Qi[0, head], Ki[0, head])
    assert np.array_equal(S.cpu().numpy(), S_ref)


# --------------------------------------------------------------------------------------
# end-to-end parity, all variants
# --------------------------------------------------------------------------------------
@pytest.mark.parametrize("B,N,h,d,heads", [(1, 64, 2, 64, None), (2, 96, 1, 64, None), (1, 256, 2, 64, None),
                                            (1, 4096, 2, 64, None), (2, 4096, 16, 64, [(0, 3), (1, 12)]),
                                            (1, 160, 2, 32, None), (1, 8192, 32, 32, [(0, 0), (0, 31)]),
                                            (2, 128, 2, 128, None), (1, 2048, 4, 128, [(0, 2)]),
                                            # the head sizes outside 32 / 64 / 128 (one-tile kernel), N = 32 included
                                            (1, 256, 2, 96, None), (1, 32, 2, 96, None), (2, 96, 1, 160, None),
                                            (1, 2048, 2, 192, [(0, 1)]), (1, 128, 2, 224, None), (1, 256, 2, 256, None)])
def test_production_qk_int32_bitexact(dev, oracle_mod, B, N, h, d, heads):
    """The int32 Q@K^T of the PRODUCTION int8 kernel, bit for bit (fa_tc_int8_b.cu:484,496,514):
    the FL_DUMP twin of the shipped schedule stores, per tile, the S^T it feeds its softmax
    (magic-biased accumulator, bias removed), its in-register int8 Q operand (quant_q_operand)
    and sQ.  Every one must equal the oracle's quantize_heads / qk_int32, and its O must equal
    flash_solve's O bit for bit (the stores do not change the computation)."""
    from quantizedmha_amd import torch_ext
    dm = h * d
    Q, K, V = rand_inputs(50 + N + h, B, N, dm)
    Q, K, V = (x.reshape(B, N, dm) for x in (Q, K, V))
    Q[0, 5, :] *= 9.0  # one outlier row: a Q group whose scale is set by a single row
    K[-1, N - 1, :d] = 0.0
    tq, tk, tv = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (Q, K, V))
    O, S, Qi, sQ = torch_ext.debug_fa_int8_dump(tq, tk, tv, dm, h)
    ref_O = torch_ext.flash_solve(tq, tk, tv, dm, h, kernel="fa_tc_int8_b")
    torch.cuda.synchronize()
    assert torch.equal(O, ref_O)
    for b, k in heads or [(b, k) for b in range(B) for k in range(h)]:
        Qi_ref, sq_ref = oracle_mod.quantize_heads(Q[b], dm, h)
        Ki_ref, _ = oracle_mod.quantize_heads(K[b], dm, h)
        assert np.array_equal(Qi[b, k].cpu().numpy(), Qi_ref[0, k]), (b, k)
        assert np.array_equal(sQ[b, k].cpu().numpy(), sq_ref[0, k]), (b, k)
        S_ref = oracle_mod.qk_int32(Qi_ref[0, k], Ki_ref[0, k])
        assert np.array_equal(S[b, k].cpu().numpy(), S_ref), (b, k)


@pytest.mark.parametrize("B,N,h,d,heads", [(1, 32, 2, 64, None), (2, 96, 1, 64, None), (1, 4096, 2, 64, None),
                                            (2, 4096, 16, 64, [(0, 3), (1, 12)]), (1, 160, 2, 32, None),
                                            (1, 8192, 32, 32, [(0, 0), (0, 31)]), (2, 128, 2, 128, None),
                                            (1, 2048, 4, 128, [(0, 2)])])
def test_production_qk_int32_bitexact_per_tensor(dev, oracle_mod, B, N, h, d, heads):
    """As test_production_qk_int32_bitexact for the per-tensor mode (fa_tc_int8_pt): the FL_DUMP twin
    of its shipped schedule stores the S^T it feeds its softmax, its in-register int8 Q operand
    (quantised with the head slice's scale) and that scale; each equals the oracle's
    quantize_heads_pt / qk_int32 bit for bit, and its O equals flash_solve's bit for bit."""
    from quantizedmha_amd import torch_ext
    dm = h * d
    Q, K, V = rand_inputs(70 + N + h, B, N, dm)
    Q, K, V = (x.reshape(B, N, dm) for x in (Q, K, V))
    Q[0, 5, :] *= 9.0  # an outlier row sets its whole head slice's scale
    K[-1, N - 1, :d] = 0.0
    tq, tk, tv = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (Q, K, V))
    O, S, Qi, sQ = torch_ext.debug_fa_int8_dump(tq, tk, tv, dm, h, per_tensor=True)
    ref_O = torch_ext.flash_solve(tq, tk, tv, dm, h, kernel="fa_tc_int8_pt")
    torch.cuda.synchronize()
    assert torch.equal(O, ref_O)
    for b, k in heads or [(b, k) for b in range(B) for k in range(h)]:
        Qi_ref, sq_ref = oracle_mod.quantize_heads_pt(Q[b], dm, h)
        Ki_ref, _ = oracle_mod.quantize_heads_pt(K[b], dm, h)
        assert np.array_equal(Qi[b, k].cpu().numpy(), Qi_ref[0, k]), (b, k)
        assert np.all(sQ[b, k].cpu().numpy() == sq_ref[0, k]), (b, k)
        S_ref = oracle_mod.qk_int32(Qi_ref[0, k], Ki_ref[0, k])
        assert np.array_equal(S[b, k].cpu().numpy(), S_ref), (b, k)


# every head size the reference's solve accepts beyond 32 / 64 / 128 (include/config.h:32: d % 32 == 0;
# round-3 VERDICT item 4); the per-tensor mode has no reference counterpart and stays at 32 / 64 / 128
OTHER_D = [96, 160, 192, 224, 256]
REF_VARIANTS = ["fa_tc_int8_b", "fa_tc_v1a", "fa", "fa_mfma", "unfused"]


@pytest.mark.parametrize("variant", REF_VARIANTS)
@pytest.mark.parametrize("d", OTHER_D)
def test_other_head_sizes_vs_oracle(dev, oracle_mod, variant, d):
    """B2 h2 N320 (10 KV groups: a partial last stage and a partial workgroup) and B1 h1 N32 (one
    group) at d = 96 ... 256 against the oracle at the variant's tolerance."""
    for B, N, h, dist in ((2, 320, 2, "normal"), (1, 32, 1, "uniform")):
        Q, K, V = rand_inputs(300 + d + N, B, N, h * d, dist)
        out = run(variant, Q, K, V, h * d, h, dev)
        ref = oracle_for(oracle_mod, variant)(Q, K, V, h * d, h)
        assert_parity(variant, out, ref)


@pytest.mark.parametrize("variant", ["fa_tc_int8_b", "fa_tc_v1a"])
@pytest.mark.parametrize("d", [96, 256])
def test_other_head_sizes_long_sequence(dev, oracle_mod, variant, d):
    """N = 2048 at d = 96 and 256 (the int8 N >= 2048 bound, 1e-4; fp16 2e-4), two heads, plus the
    per-tensor mode refusing these head sizes with a NOSYS status instead of running."""
    from quantizedmha_amd import torch_ext
    Q, K, V = rand_inputs(900 + d, 1, 2048, 2 * d)
    out = run(variant, Q, K, V, 2 * d, 2, dev)
    ref = oracle_for(oracle_mod, variant)(Q, K, V, 2 * d, 2)
    assert_parity(variant, out, ref)
    with pytest.raises(RuntimeError, match="not supported"):
        torch_ext.flash_solve(*(torch.from_numpy(x).to(dev) for x in (Q, K, V)), 2 * d, 2, kernel="fa_tc_int8_pt")


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("case", ["medium", "large"])
def test_variant_vs_reference_golden(dev, oracle_mod, variant, case):
    N, dm, h, Q, K, V, O = load_case(case)
    out = run(variant, Q, K, V, dm, h, dev)
    assert np.isfinite(out).all()
    ref = oracle_for(oracle_mod, variant)(Q, K, V, dm, h)
    assert_parity(variant, out, ref)
    e_gold = np.abs(out - O).max()
    assert e_gold <= TOL_GOLDEN[variant], e_gold


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("B,N,d_model,h,dist", [
    (1, 32, 32, 1, "normal"),     # single group, d=32
    (2, 96, 128, 2, "normal"),    # N/32 = 3: partial workgroup and partial KV stage
    (1, 160, 256, 2, "uniform"),  # d=128, U[0,1) (the reference's profiling distribution)
    (3, 256, 128, 2, "uniform"),  # batch
    (1, 1024, 64, 1, "normal"),   # longer sequence
    (2, 608, 96, 3, "normal"),    # d=32, N/32 = 19: ring period 6 + a remainder, partial workgroup
    (1, 416, 256, 2, "normal"),   # d=128, N/32 = 13
])
def test_variant_vs_oracle_random(dev, oracle_mod, variant, B, N, d_model, h, dist):
    Q, K, V = rand_inputs(10 + N + B, B, N, d_model, dist)
    out = run(variant, Q, K, V, d_model, h, dev)
    ref = oracle_for(oracle_mod, variant)(Q, K, V, d_model, h)
    assert_parity(variant, out, ref)


def _sweep_shapes(seed, n):
    """n random (B, N, H, d) with N a multiple of 32 from 32 to 2048 (odd group counts
    included), d in {32, 64, 128}, H in 1..8, B in 1..5, sized so the oracle finishes fast."""
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        d = int(rng.choice([32, 64, 128]))
        G = int(rng.integers(1, 65))
        H = int(rng.integers(1, 9))
        B = int(rng.integers(1, 6))
        if B * H * (32 * G) ** 2 * d > 2e9:
            continue
        out.append((B, 32 * G, H, d))
    return out


@pytest.mark.parametrize("variant", VARIANTS)
def test_random_shape_sweep(dev, oracle_mod, variant):
    """Property sweep: 10 random shapes per variant (every d, odd and even KV-group counts, batch
    and head counts) against the oracle at the variant's tolerance."""
    for i, (B, N, H, d) in enumerate(_sweep_shapes(77 + VARIANTS.index(variant), 10)):
        Q, K, V = rand_inputs(1000 + i, B, N, H * d, "normal" if i % 2 else "uniform")
        out = run(variant, Q, K, V, H * d, H, dev)
        ref = oracle_for(oracle_mod, variant)(Q, K, V, H * d, H)
        try:
            assert_parity(variant, out, ref)
        except AssertionError as e:
            raise AssertionError(f"{variant} B{B} N{N} H{H} d{d}: {e}") from None


# bound against exact (fp64) attention at N = 65536: each output averages thousands of keys, so
# the quantisation / rounding errors average out far below the short-sequence budgets (int8 5e-3,
# fp16 1e-3); first run on MI355X: int8 7.3e-5, per-tensor 9.6e-5, fp16 2.1e-6, fp32 <= 6.7e-8
TOL_FP64 = {"fa_tc_int8_b": 1e-3, "fa_tc_int8_pt": 1e-3, "fa_tc_v1a": 1e-4, "fa": 1e-6, "fa_mfma": 1e-6,
            "unfused": 1e-6}


@pytest.mark.parametrize("variant", VARIANTS)
def test_maximum_sequence_length_sampled_rows(dev, variant):
    """N = 65536 (unfused: 16384 -- its N x N score buffer), two heads of d = 64: 2048 KV tiles
    per sweep, far past every other test.  The CPU oracles are O(N^2 d) per head and too slow at
    this length, so 96 query rows spread over the sequence (first and last rows included) are
    checked against exact fp64 attention within each variant's error budget, and every output
    must be a convex combination of V (inside [min V, max V] of its head)."""
    N = 16384 if variant == "unfused" else 65536
    dm, h = 128, 2
    d = dm // h
    Q, K, V = rand_inputs(2024, 1, N, dm)
    out = run(variant, Q, K, V, dm, h, dev)
    assert np.isfinite(out).all()
    rows = np.unique(np.concatenate([np.linspace(0, N - 1, 94).astype(int), [1, N - 2]]))
    err = 0.0
    for k in range(h):
        c = slice(k * d, (k + 1) * d)
        Vk = V[:, c].astype(np.float64)
        assert out[:, c].min() >= Vk.min() - 1e-4 and out[:, c].max() <= Vk.max() + 1e-4
        S = Q[rows, c].astype(np.float64) @ K[:, c].astype(np.float64).T / np.sqrt(d)
        P = np.exp(S - S.max(axis=1, keepdims=True))
        ref = (P / P.sum(axis=1, keepdims=True)) @ Vk
        err = max(err, float(np.abs(out[rows, c] - ref).max()))
    parity_log.record("test_maximum_sequence_length_sampled_rows", variant + " (vs fp64)", err, 0.0,
                      TOL_FP64[variant])
    assert err <= TOL_FP64[variant], (variant, err)


@pytest.mark.parametrize("variant", VARIANTS)
def test_all_ones_driver_check(dev, oracle_mod, variant):
    """drivers/main.cu:73-101: all-ones input, every output 1.0 within max(1e-3, 1e-3*|ref|)."""
    ones = np.ones((128, 128), np.float32)
    out = run(variant, ones, ones, ones, 128, 2, dev)
    assert oracle_mod.verify_results(out, ones) == -1


@pytest.mark.parametrize("variant", VARIANTS)
def test_edge_values(dev, oracle_mod, variant):
    N, dm, h = 128, 128, 2
    rng = np.random.default_rng(99)
    Q = np.zeros((N, dm), np.float32)  # zero scores: uniform average, alpha == 1 everywhere
    K = (rng.standard_normal((N, dm)) * 3).astype(np.float32)
    V = (rng.standard_normal((N, dm))).astype(np.float32)
    out = run(variant, Q, K, V, dm, h, dev)
    ref = oracle_for(oracle_mod, variant)(Q, K, V, dm, h)
    assert_parity(variant, out, ref)
    # a spike: one key far above the rest forces a large running-max jump mid-sequence
    Q = (rng.standard_normal((N, dm)) * 0.5).astype(np.float32)
    K = (rng.standard_normal((N, dm)) * 0.5).astype(np.float32)
    K[77] = Q[3] * 8
    out = run(variant, Q, K, V, dm, h, dev)
    ref = oracle_for(oracle_mod, variant)(Q, K, V, dm, h)
    assert_parity(variant, out, ref, scale=4)


@pytest.mark.parametrize("variant", VARIANTS)
def test_growing_scores_reanchor(dev, oracle_mod, variant):
    """Scores that climb by ~100 log2 units along the sequence: every tile raises the running
    max, and the int8 kernel's anchored accumulator must re-anchor (m - anchor > 48)."""
    N, dm, h = 512, 128, 2
    rng = np.random.default_rng(7)
    Q = (rng.standard_normal((N, dm)) * 0.2 + 1.0).astype(np.float32)
    ramp = np.linspace(0.0, 4.0, N, dtype=np.float32)[:, None]
    K = ((rng.standard_normal((N, dm)) * 0.2 + 1.0) * ramp).astype(np.float32)
    V = rng.standard_normal((N, dm)).astype(np.float32)
    out = run(variant, Q, K, V, dm, h, dev)
    ref = oracle_for(oracle_mod, variant)(Q, K, V, dm, h)
    # fp16: with a few dominant keys per row one exp2-vs-expf ulp can flip half(p) (2^-11
    # relative) and move O by ~5e-4 |V|; bound by the reference's own 1e-3 verify tolerance.
    # (fa_tc_int8_pt ran at 5x too until r06: its oracle's nats score constant flipped Pi on these
    # 50-unit scores; the base-2 restatement of the kernel's constant agrees to 5e-7)
    assert_parity(variant, out, ref, scale=5.0 if variant == "fa_tc_v1a" else 1.0)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("d", [32, 64, 128])
def test_large_first_tile_and_spike_no_overflow(dev, oracle_mod, variant, d):
    """Running-max jumps far beyond the int8 kernel's 48-log2 anchor headroom in ONE tile.

    (1) constant Q = K = 3.5: every score is 3.5^2 * sqrt(d) (98 nats at d = 64, ~141 log2
    units above m0 = 0) already in the first tile; the reference returns mean(V) per head.
    (2) a single key tile whose scores sit ~200 log2 units above the rest mid-sequence.
    Before the fix the shift 2^(m_new - anchor) overflowed to inf, the re-anchor made it NaN
    and the epilogue's l > 1e-20 guard silently wrote 0 (round-1 ADVICE, qmha_fa_int8.hip:728)."""
    N, h = 256, 2
    dm = d * h
    rng = np.random.default_rng(40 + d)
    Q = np.full((N, dm), 3.5, np.float32)
    K = np.full((N, dm), 3.5, np.float32)
    V = rng.standard_normal((N, dm)).astype(np.float32)
    out = run(variant, Q, K, V, dm, h, dev)
    ref = oracle_for(oracle_mod, variant)(Q, K, V, dm, h)
    assert np.isfinite(out).all()
    assert np.abs(ref - V.mean(axis=0, keepdims=True)).max() <= 5e-2  # the oracle really averages V
    assert_parity(variant, out, ref)
    # spike: keys 160..191 (one 32-key tile) strongly aligned with every query
    Q = (rng.standard_normal((N, dm)) * 0.3 + 1.0).astype(np.float32)
    K = (rng.standard_normal((N, dm)) * 0.3).astype(np.float32)
    K[160:192] = 6.0
    out = run(variant, Q, K, V, dm, h, dev)
    ref = oracle_for(oracle_mod, variant)(Q, K, V, dm, h)
    assert np.isfinite(out).all() and np.abs(out).max() > 0.01
    assert_parity(variant, out, ref, scale=5.0 if variant == "fa_tc_v1a" else 1.0)


@pytest.mark.parametrize("variant", ["fa_tc_int8_b", "fa_tc_v1a", "fa"])
def test_underflow_guard_and_zero_v(dev, oracle_mod, variant):
    """m0 = 0 (fa_tc_int8_b.cu:402): with all scores far below 0 the row sum underflows past the
    guard (1e-20 int8, 1e-10 fp16/fp32, fa_tc_int8_b.cu:549-553) and the reference writes 0.
    (The unfused path runs a max-subtracted row softmax, unfused.cu, and has no such guard.)"""
    N, dm, h = 128, 128, 2
    rng = np.random.default_rng(8)
    Q = np.full((N, dm), 3.0, np.float32)
    K = np.full((N, dm), -3.0, np.float32) + (rng.standard_normal((N, dm)) * 0.01).astype(np.float32)
    V = rng.standard_normal((N, dm)).astype(np.float32)
    out = run(variant, Q, K, V, dm, h, dev)
    ref = oracle_for(oracle_mod, variant)(Q, K, V, dm, h)
    assert np.array_equal(ref, np.zeros_like(ref))  # the oracle takes the guard
    assert np.array_equal(out, np.zeros_like(out))
    # V == 0: any finite attention is exactly 0
    Q, K = (rng.standard_normal((N, dm)).astype(np.float32) for _ in range(2))
    out = run(variant, Q, K, np.zeros((N, dm), np.float32), dm, h, dev)
    assert np.array_equal(out, np.zeros_like(out))


def test_deterministic(dev):
    Q, K, V = rand_inputs(5, 2, 512, 256)
    a = run("fa_tc_int8_b", Q, K, V, 256, 4, dev)
    b = run("fa_tc_int8_b", Q, K, V, 256, 4, dev)
    assert np.array_equal(a, b)


def test_c_abi_solve_per_variant_libraries(dev, oracle_mod):
    """Bind `solve` from each libqmha_<variant>.so exactly as a reference caller would."""
    N, dm, h = 128, 256, 4
    Q, K, V = rand_inputs(21, 1, N, dm)
    tq, tk, tv = (torch.from_numpy(x).to(dev) for x in (Q, K, V))
    for variant in VARIANTS:
        lib = ctypes.CDLL(os.path.join(ROOT, "quantizedmha_amd", "lib", f"libqmha_{variant}.so"))
        lib.solve.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3
        lib.solve.restype = None
        out = torch.empty_like(tq)
        lib.solve(tq.data_ptr(), tk.data_ptr(), tv.data_ptr(), out.data_ptr(), N, dm, h)
        ref = oracle_for(oracle_mod, variant)(Q, K, V, dm, h)
        assert_parity(variant, out.cpu().numpy(), ref)


def test_jax_ext_raw_pointer_entry(dev, oracle_mod):
    from quantizedmha_amd import jax_ext
    N, dm, h = 64, 128, 2
    Q, K, V = rand_inputs(31, 1, N, dm)
    tq, tk, tv = (torch.from_numpy(x).to(dev) for x in (Q, K, V))
    out = torch.empty_like(tq)
    jax_ext.flash_solve(tq.data_ptr(), tk.data_ptr(), tv.data_ptr(), out.data_ptr(), N, dm, h, "fa_tc_v1a")
    ref = oracle_mod.fa_fp16(Q, K, V, dm, h)
    assert np.abs(out.cpu().numpy() - ref).max() <= TOL_ORACLE["fa_tc_v1a"]


def _slices_vs_oracle(oracle_fn, Q, K, V, out, d, slices, nthreads=16):
    """Stack the (batch, head) slices as the heads of one [N, S*d] problem, run the oracle on
    them in one multi-threaded call and return (gpu, oracle) as [N, S*d] arrays."""
    def stack(x):
        host = (lambda t: t.cpu().numpy()) if isinstance(x, torch.Tensor) else (lambda t: t)
        return np.concatenate([host(x[b, :, k * d:(k + 1) * d]) for b, k in slices], axis=1)
    q, kk, v, o = (stack(x) for x in (Q, K, V, out))
    ref = oracle_fn(q, kk, v, len(slices) * d, len(slices), nthreads)
    return o, ref


# 16 (batch, head) slices of a 16 x 16 grid, one per batch element, heads spread so that the
# workgroups they map to fall on all 8 XCDs through the launcher's block remap
C_SLICES = [(b, (7 * b + 3) % 16) for b in range(16)]


def _all_slices_vs_oracle(oracle_fn, Q, K, V, out, d, slices=None, per_call=16):
    """Every (batch, head) slice (or the given ones) of a [B, N, H*d] call against the oracle,
    per_call slices per multi-threaded oracle call (16 threads: the GPU box's CPU share); returns
    (gpu, oracle) stacked as [calls, N, per_call*d] arrays for one assert_parity."""
    B, H = Q.shape[0], Q.shape[2] // d
    if slices is None:  # the whole call: one device -> host copy per tensor
        Q, K, V, out = (x.cpu().numpy() for x in (Q, K, V, out))
        slices = [(b, k) for b in range(B) for k in range(H)]
    got, ref = [], []
    for i in range(0, len(slices), per_call):
        g, r = _slices_vs_oracle(oracle_fn, Q, K, V, out, d, slices[i:i + per_call])
        got.append(g)
        ref.append(r)
    return np.stack(got), np.stack(ref)


@pytest.mark.parametrize("variant", INT8_VARIANTS)
@pytest.mark.parametrize("B,H,d", [(16, 8, 128), (16, 32, 32)])
def test_int8_other_head_sizes_bench_shapes(dev, oracle_mod, variant, B, H, d):
    """The d = 128 and d = 32 shapes DESIGN.md quotes timings for (N = 4096, B16 H8 d128 and
    B16 H32 d32, both int8 variants): 8 (batch, head) slices spread over the grid against the
    oracle at the N >= 2048 bound, all outputs finite."""
    from quantizedmha_amd import torch_ext
    N = 4096
    g = torch.Generator(device=dev).manual_seed(d)
    Q, K, V = (torch.randn(B, N, H * d, device=dev, generator=g) * 0.5 for _ in range(3))
    out = torch_ext.flash_solve(Q, K, V, H * d, H, kernel=variant)
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    slices = [(2 * i, (5 * i + 1) % H) for i in range(8)]
    oracle_fn = oracle_mod.fa_int8 if variant == "fa_tc_int8_b" else oracle_mod.fa_int8_pt
    got, ref = _slices_vs_oracle(oracle_fn, Q, K, V, out, d, slices)
    assert_parity(variant, got, ref)


def test_full_baseline_config_all_heads(dev, oracle_mod):
    """BASELINE C4 (B16 H16 N4096 d64, int8): the whole call on the GPU, ALL 256 (batch, head)
    slices against the oracle at the N >= 2048 bound (round-3 VERDICT: full coverage, not 16
    samples), every row's convexity (all-positive V => outputs inside [0, 1]) everywhere."""
    from quantizedmha_amd import torch_ext
    B, N, H, d = 16, 4096, 16, 64
    g = torch.Generator(device=dev).manual_seed(0)
    Q = torch.randn(B, N, H * d, device=dev, generator=g) * 0.5
    K = torch.randn(B, N, H * d, device=dev, generator=g) * 0.5
    V = torch.rand(B, N, H * d, device=dev, generator=g)
    out = torch_ext.flash_solve(Q, K, V, H * d, H, kernel="fa_tc_int8_b")
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    assert float(out.min()) >= 0.0 and float(out.max()) <= 1.0
    got, ref = _all_slices_vs_oracle(oracle_mod.fa_int8, Q, K, V, out, d)
    assert got.shape == (16, N, 16 * d)
    assert_parity("fa_tc_int8_b", got, ref, N=N)
    # the reference's calling pattern, one sequence per call: a one-round grid, which the launcher
    # runs with issue-priority fairness -- scheduling only, so every sequence must
    # come out bit-identical to its slice of the batched (10.7-round, fairness off) launch
    for b in (0, 7, 15):
        one = torch_ext.flash_solve(Q[b], K[b], V[b], H * d, H, kernel="fa_tc_int8_b")
        torch.cuda.synchronize()
        assert torch.equal(one, out[b]), b


def test_reference_own_config_int8_all_heads(dev, oracle_mod):
    """The reference's own compiled configuration (include/config.h:22-28: N=8192, d_model=1024,
    h=32 -> d=32; the shape of its README.md:19 timing) through fa_tc_int8_b: ALL 32 heads against
    the oracle at 1e-4, U[0,1) inputs (the reference's data.cu:16-22 distribution)."""
    from quantizedmha_amd import torch_ext
    N, H, d = 8192, 32, 32
    g = torch.Generator(device=dev).manual_seed(8192)
    Q, K, V = (torch.rand(1, N, H * d, device=dev, generator=g) for _ in range(3))
    out = torch_ext.flash_solve(Q, K, V, H * d, H, kernel="fa_tc_int8_b")
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    got, ref = _all_slices_vs_oracle(oracle_mod.fa_int8, Q, K, V, out, d)
    assert got.shape == (2, N, 16 * d)
    assert_parity("fa_tc_int8_b", got, ref, N=N)


def test_c5_global_batch_on_one_gpu(dev, oracle_mod):
    """BASELINE C5's whole global batch (B=128 H16 N4096 d64, 8 GPUs x 16 in the driver's scaling
    run) through one launch on one GPU, via the batch-shard entry point at world 1: a 65,536-
    workgroup grid over 8.6 GB per tensor.  Sequences spread over the batch (so over the workspace
    and the XCD remap) against the oracle; every output finite and inside [0, 1] (V in [0, 1))."""
    from quantizedmha_amd.shard import solve_sharded
    B, N, H, d = 128, 4096, 16, 64
    g = torch.Generator(device=dev).manual_seed(128)
    Q = torch.randn(B, N, H * d, device=dev, generator=g) * 0.5
    K = torch.randn(B, N, H * d, device=dev, generator=g) * 0.5
    V = torch.rand(B, N, H * d, device=dev, generator=g)
    out = solve_sharded(Q, K, V, H * d, H, "fa_tc_int8_b")
    torch.cuda.synchronize()
    assert out.shape == (B, N, H * d)
    assert bool(torch.isfinite(out).all()) and float(out.min()) >= 0.0 and float(out.max()) <= 1.0
    # 64 slices: every other sequence of the 128 (the whole batch range, so every part of the
    # workspace and of the XCD remap), heads rotating through all 16
    slices = [(b, (5 * b + 3) % H) for b in range(0, B, 2)]
    got, ref = _all_slices_vs_oracle(oracle_mod.fa_int8, Q, K, V, out, d, slices)
    assert got.shape[0] * got.shape[2] // d == 64
    assert_parity("fa_tc_int8_b", got, ref, N=N)
    del Q, K, V, out
    torch.cuda.empty_cache()


def fp16_lazy_tol(N):
    """GPU vs its own contract (oracle fa_fp16_lazy): v_exp_f32 vs libm exp2f ulps flip a half(p) rounding,
    which moves a row by 2^-11 of that key's weight; short rows give one key a large weight (observed 5.1e-5
    at N = 32 in the r06 sweep, <= 1.5e-5 from N = 256 on)."""
    return 1e-4 if N <= 256 else 4e-5


@pytest.mark.parametrize("N,d", [(32, 64), (64, 32), (96, 128), (256, 64), (1024, 64), (2048, 128), (4096, 32)])
@pytest.mark.parametrize("dist", ["normal", "uniform"])
def test_fp16_lazy_base_contract(dev, oracle_mod, N, d, dist):
    """The fp16 kernel's lazy softmax base (r06): pinned tightly to its own restatement
    (oracle fa_fp16_lazy) and held to the 2e-4 fp16 bound against the reference's algorithm (fa_fp16)."""
    h = 2
    Q, K, V = rand_inputs(300 + N + d, 2, N, h * d, dist)
    out = run("fa_tc_v1a", Q, K, V, h * d, h, dev)
    lazy = oracle_mod.fa_fp16_lazy(Q, K, V, h * d, h)
    err = float(np.abs(out.astype(np.float64) - lazy).max())
    parity_log.record(f"test_fp16_lazy_base_contract[{N}-{d}-{dist}]", "fa_tc_v1a (vs lazy)", err, 0.0, fp16_lazy_tol(N))
    assert err <= fp16_lazy_tol(N), err
    assert_parity("fa_tc_v1a", out, oracle_mod.fa_fp16(Q, K, V, h * d, h))


@pytest.mark.parametrize("variant,cap", [("fa_tc_int8_pt", 2047.0 / 127.0), ("fa_tc_v1a", 4096.0)])
@pytest.mark.parametrize("d", [32, 64, 128])
def test_lazy_base_staircase(dev, oracle_mod, variant, cap, d):
    """The lazy softmax base near its cap (r06; a row's base moves only when the p of
    one of its key halves sum above the cap: 2047/127 per-tensor, 2^12 fp16).  In every 32-key tile two
    keys -- one per lane half -- score 0.95 log2(cap) log2 units above the previous tile's, the other 30
    sit 8 units below them, so a half sums just under the cap on every other tile (the per-tensor Pi reach
    ~1800 of the 2047 an f16 subnormal holds, the fp16 P ~3800) and the base moves on the next.  Checked
    against the kernel's own contract (the per-tensor oracle is lazy; oracle fa_fp16_lazy) and, for fp16,
    against the reference's algorithm."""
    B, N, h = 2, 512, 2
    dm = h * d
    rng = np.random.default_rng(int(cap) + d)
    Q = (0.5 + 0.01 * rng.standard_normal((B, N, dm))).astype(np.float32)
    # log2-unit score of a key at level a: 0.5 * a * d / sqrt(d) * log2(e)
    unit = 1.0 / (0.5 * np.sqrt(d) * np.log2(np.e))
    hi = np.arange(N // 32) * 0.95 * np.log2(cap) * unit
    level = np.repeat(hi, 32) - 8.0 * unit
    level[0::32] = hi  # key 0 of each tile (lane half 0) and key 4 (half 1) lead their tile
    level[4::32] = hi
    K = (level[None, :, None] + 0.01 * rng.standard_normal((B, N, dm))).astype(np.float32)
    V = rng.standard_normal((B, N, dm)).astype(np.float32)
    out = run(variant, Q, K, V, dm, h, dev)
    if variant == "fa_tc_int8_pt":
        assert_parity(variant, out, oracle_mod.fa_int8_pt(Q, K, V, dm, h))
        return
    # Two dominant keys per row with p ~ 2^11.4 (the reference's dominant p is 1, exact in half): a ~1e-5
    # log2-unit score difference from the MFMA's fp32 summation order flips half(p) of a dominant key
    # (one half ulp: at most 2^-10 relative) and moves the row by up to 2^-10 max|V| (observed 1.4e-3 against
    # fa_fp16_lazy, with max|V| = 4.4).  So
    # the criteria here: as accurate as the reference's algorithm against exact attention, and within that
    # flip bound of the kernel's own contract
    exact = oracle_mod.cpu_attention(Q, K, V, dm, h)
    e_gpu = float(np.abs(out.astype(np.float64) - exact).max())
    e_ref = float(np.abs(oracle_mod.fa_fp16(Q, K, V, dm, h).astype(np.float64) - exact).max())
    parity_log.record(f"test_lazy_base_staircase[{variant}-{d}]", "fa_tc_v1a (vs fp32 attn)", e_gpu, 0.0, 1.1 * e_ref)
    assert e_gpu <= 1.1 * e_ref, (e_gpu, e_ref)
    lazy = oracle_mod.fa_fp16_lazy(Q, K, V, dm, h)
    err = float(np.abs(out.astype(np.float64) - lazy).max())
    tol = 2.0 ** -10 * float(np.abs(V).max())
    parity_log.record(f"test_lazy_base_staircase[{variant}-{d}]", "fa_tc_v1a (vs lazy)", err, 0.0, tol)
    assert err <= tol, (err, tol)


def test_c3_fp16_full_config_all_heads(dev, oracle_mod):
    """BASELINE C3 (fa_tc_v1a, fp16 MFMA, B16 H16 N4096 d64) at its own workload: the whole
    call on the GPU, ALL 256 (batch, head) slices against oracle fa_fp16 at 2e-4 (fa_tc_v1a.cu:222-413)."""
    from quantizedmha_amd import torch_ext
    B, N, H, d = 16, 4096, 16, 64
    g = torch.Generator(device=dev).manual_seed(33)
    Q, K, V = (torch.randn(B, N, H * d, device=dev, generator=g) * 0.5 for _ in range(3))
    out = torch_ext.flash_solve(Q, K, V, H * d, H, kernel="fa_tc_v1a")
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    got, ref = _all_slices_vs_oracle(oracle_mod.fa_fp16, Q, K, V, out, d)
    assert_parity("fa_tc_v1a", got, ref, N=N)


@pytest.mark.parametrize("variant", ["fa", "fa_mfma"])
def test_c2_fp32_full_config_all_heads(dev, oracle_mod, variant):
    """BASELINE C2 (fa, fp32, B8 H8 N1024 d64) at its own workload, every one of the 64 heads
    against oracle fa_fp32 at 1e-5 (fa.cu:211-400): the scalar no-matrix-core kernel the config
    names (fa) and its fp32-MFMA sibling (fa_mfma)."""
    from quantizedmha_amd import torch_ext
    B, N, H, d = 8, 1024, 8, 64
    g = torch.Generator(device=dev).manual_seed(22)
    Q, K, V = (torch.randn(B, N, H * d, device=dev, generator=g) * 0.5 for _ in range(3))
    out = torch_ext.flash_solve(Q, K, V, H * d, H, kernel=variant)
    torch.cuda.synchronize()
    ref = oracle_mod.fa_fp32(Q.cpu().numpy(), K.cpu().numpy(), V.cpu().numpy(), H * d, H, 16)
    assert_parity(variant, out.cpu().numpy(), ref)


def test_compiled_torch_ext_module(dev, oracle_mod):
    """The compiled pybind module (quantizedmha_amd/csrc/torch_ext.cpp, the reference's
    extensions/torch/torch_ext.cpp drop-in): `import torch_ext; torch_ext.flash_solve(...)`
    unchanged, bit-identical to the ctypes mirror for every variant, 2-D and 3-D inputs,
    the reference's errors and its unknown-kernel warning."""
    import sys
    import warnings
    sys.path.insert(0, os.path.join(ROOT, "quantizedmha_amd", "lib"))
    try:
        import torch_ext as compiled
    finally:
        sys.path.pop(0)
    from quantizedmha_amd import torch_ext as mirror
    Q, K, V = (torch.from_numpy(x).to(dev) for x in rand_inputs(44, 2, 256, 256))
    for variant in VARIANTS:
        a = compiled.flash_solve(Q, K, V, 256, 4, variant)
        b = mirror.flash_solve(Q, K, V, 256, 4, kernel=variant)
        torch.cuda.synchronize()
        assert torch.equal(a, b), variant
    two_d = compiled.flash_solve(Q[1], K[1], V[1], 256, 4)  # reference form: [N, d_model], default kernel
    assert torch.equal(two_d, mirror.flash_solve(Q, K, V, 256, 4)[1])
    ref = oracle_mod.fa_int8(Q[1].cpu().numpy(), K[1].cpu().numpy(), V[1].cpu().numpy(), 256, 4)
    assert_parity("fa_tc_int8_b", two_d.cpu().numpy(), ref)
    with pytest.raises(RuntimeError, match="Inputs must be CUDA tensors"):
        compiled.flash_solve(Q.cpu(), K, V, 256, 4)
    with pytest.raises(RuntimeError, match="Q must be float32"):
        compiled.flash_solve(Q.double(), K, V, 256, 4)
    with pytest.raises(RuntimeError, match="divisible by d_model"):
        compiled.flash_solve(Q, K, V, 255, 4)
    with warnings.catch_warnings(record=True):
        warnings.simplefilter("always")
        c = compiled.flash_solve(Q, K, V, 256, 4, "fa_tc_v2b")  # unknown -> warned, default kernel
    assert torch.equal(c, mirror.flash_solve(Q, K, V, 256, 4))
    # malformed 3-D shapes (round-2 ADVICE): both front-ends read a non-[B, N, d_model] 3-D tensor
    # as ONE sequence of numel/d_model rows, like the reference, and reject mismatched K / V shapes
    nhd = [x[1].reshape(256, 4, 64) for x in (Q, K, V)]  # [N, h, d]
    for fe in (compiled.flash_solve, mirror.flash_solve):
        r = fe(*nhd, 256, 4)
        torch.cuda.synchronize()
        assert r.shape == (256, 4, 64) and torch.equal(r.reshape(256, 256), two_d)
        with pytest.raises(RuntimeError, match="same shape"):
            fe(Q, K[:, :128], V, 256, 4)
        with pytest.raises(RuntimeError, match="same shape"):
            fe(Q[1].reshape(256, 4, 64), K[1], V[1], 256, 4)
    small = Q[0, :64].reshape(32, 64, 8).contiguous()  # last dim != d_model: one sequence of 2 rows
    with pytest.raises(RuntimeError, match="multiple of 32"):
        compiled.flash_solve(small, small, small, 1024, 16)
    with pytest.raises(RuntimeError, match="multiple of 32"):
        mirror.flash_solve(small, small, small, 1024, 16)


def test_driver_binary_end_to_end(dev, tmp_path):
    exe = os.path.join(ROOT, "quantizedmha_amd", "bin", "qmha_profile")
    for kernel in VARIANTS:
        r = subprocess.run([exe, f"--kernel={kernel}", "--N=256", "--d_model=128", "--h=2", "--B=2", "--warmup=1",
                            "--runs=2", "--check-random", "--json", f"--cache-dir={tmp_path}"],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "Correctness check PASSED" in r.stdout
        assert '"check_random": "passed"' in r.stdout


@pytest.mark.parametrize("variant", VARIANTS)
def test_solve_ws_caller_scratch_and_graph_capture(dev, variant):
    """qmha_solve_ws (caller-owned scratch, no allocation or synchronisation inside): equal to
    qmha_solve_ex bit for bit on a side stream, and capturable in a HIP graph (torch.cuda.CUDAGraph
    on ROCm) whose replays follow new inputs written into the captured buffers."""
    from quantizedmha_amd import _lib, torch_ext
    lib = _lib.load()
    B, N, H, d = 2, 1024, 8, 64
    g = torch.Generator(device=dev).manual_seed(9)
    Q, K, V = (torch.randn(B, N, H * d, device=dev, generator=g) * 0.5 for _ in range(3))
    vid = _lib.variant_id(variant)
    ws_bytes = lib.qmha_workspace_size(B, N, H * d, H, vid)
    ws = torch.empty(max(ws_bytes, 256), dtype=torch.uint8, device=dev)

    def call(out, stream):
        st = lib.qmha_solve_ws(Q.data_ptr(), K.data_ptr(), V.data_ptr(), out.data_ptr(), B, N, H * d, H, vid,
                               ws.data_ptr(), ws_bytes, stream.cuda_stream)
        _lib.check(st, variant)

    ref = torch_ext.flash_solve(Q, K, V, H * d, H, kernel=variant)
    torch.cuda.synchronize()
    O = torch.empty_like(Q)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        call(O, side)
    side.synchronize()
    assert torch.equal(O, ref)
    if ws_bytes:  # too small a workspace is refused, not overrun
        st = lib.qmha_solve_ws(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), B, N, H * d, H, vid,
                               ws.data_ptr(), ws_bytes - 1, side.cuda_stream)
        assert st != 0
    O2 = torch.zeros_like(Q)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        call(O2, torch.cuda.current_stream(dev))
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(O2, ref)
    Q.mul_(0.75)
    V.add_(0.25)
    ref2 = torch_ext.flash_solve(Q, K, V, H * d, H, kernel=variant)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(O2, ref2) and not torch.equal(ref2, ref)


@pytest.mark.parametrize("variant", ["fa_tc_int8_b", "fa_tc_v1a"])
def test_overlap_chunks_bit_identical(dev, variant):
    """Batch-chunked pre-pass/main overlap (qmha_set_overlap_chunks) must not change a bit, and
    two calls in a row on the same workspace must agree (catches LDS-DMA / stream races)."""
    from quantizedmha_amd import _lib, torch_ext
    lib = _lib.load()
    B, N, H, d = 8, 1024, 16, 64
    g = torch.Generator(device=dev).manual_seed(3)
    Q, K, V = (torch.randn(B, N, H * d, device=dev, generator=g) * 0.5 for _ in range(3))
    prev = lib.qmha_set_overlap_chunks(1)
    try:
        ref = torch_ext.flash_solve(Q, K, V, H * d, H, kernel=variant)
        for chunks in (2, 4):
            lib.qmha_set_overlap_chunks(chunks)
            for _ in range(2):
                out = torch_ext.flash_solve(Q, K, V, H * d, H, kernel=variant)
                assert torch.equal(out, ref), (variant, chunks)
    finally:
        lib.qmha_set_overlap_chunks(prev)
