"""The fused per-block int8 call (FL_FUSED): one kernel quantises K / V itself, its workgroups
producing K / V groups for each other under agent-coherent stores and per-group flags.  Its output must equal
the two-launch path (pre-pass, then the same sweep) bit for bit.

The checks are built so that a consumer reading a stale or not-yet-landed line CAN fail them (round-4
VERDICT, weak #3): before a fused call the scratch it reads holds either a random poison pattern or the
bytes of a DIFFERENT input set, never the bytes the call is about to produce.

In a file of its own that sorts after every other GPU test file, so that a failure of this path cannot stop
the rest of a `pytest -x -m gpu` run."""
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from quantizedmha_amd import _lib
    _lib.load()  # raises if the HIP library is missing: no silent fallback
    return torch.device("cuda:0")


SHAPES = [(2, 1024, 8, 64), (4, 4096, 16, 64), (16, 4096, 16, 64), (1, 8192, 32, 32), (2, 512, 8, 32),
          (2, 2048, 4, 128), (8, 4096, 8, 128), (3, 96, 2, 64), (5, 2080, 3, 64), (1, 65536, 1, 64)]


F16_SHAPES = [(2, 1024, 8, 64), (4, 4096, 16, 64), (16, 4096, 16, 64), (1, 8192, 32, 32), (2, 2048, 4, 128),
              (3, 96, 2, 64), (5, 2080, 3, 64), (1, 65536, 1, 64)]


@pytest.mark.parametrize("variant,B,N,H,d", [("fa_tc_int8_b",) + s for s in SHAPES] + [("fa_tc_v1a",) + s for s in F16_SHAPES])
def test_fused_bit_identical(dev, variant, B, N, H, d):
    """Three input sets X0, X1, X2; references from the two-launch path (mode 0).  Then, with the fused call:
      1. a caller-owned workspace (qmha_solve_ws) filled with random bytes before each call, for each set;
      2. back-to-back calls X0, X1, X2, X0 on that workspace without refilling: each call's scratch holds
         the previous set's bytes;
      3. the library's own workspace, which the reference calls left holding X2's bytes: X0, X1;
      4. every wave producing its own head after a zero wait bound (the fallback path), poisoned workspace;
      5. the cross-XCD test rule (every group produced by a workgroup of another XCD; on grids of more
         than one round of workgroups some consumers outwait it and produce for themselves), poisoned
         workspace, sets X1 and X2.
    Shapes: small / one-round / C4 (10.7 rounds) at d = 64, the reference's (2 rounds at d = 32), d = 32 and
    d = 128 one- and multi-round, N = 96 (one q-block), a ragged grid whose heads straddle the XCD ranges and
    rounds (B5 H3 N2080), and one head longer than a round (N = 65536: routed to the two launches,
    tests/test_fused_schedule.py).  The fp16 call (fa_tc_v1a, K / V converted inside the sweep with the same
    split and flags) the same way, without step 4 (its wait bound is fixed)."""
    from quantizedmha_amd import _lib
    lib = _lib.load()
    vid = _lib.variant_id(variant)
    is8 = variant == "fa_tc_int8_b"
    set_fused = lib.qmha_debug_set_int8_fused if is8 else lib.qmha_debug_set_f16_fused
    dm = H * d
    stream = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev).manual_seed(31 + N + B)
    sets = [tuple(torch.randn(B, N, dm, device=dev, generator=g) * (0.5 + 0.25 * i) for _ in range(3)) for i in range(3)]

    def call(i, ws=None):
        Q, K, V = sets[i]
        O = torch.full_like(Q, float("nan"))
        if ws is None:
            _lib.check(lib.qmha_solve_ex(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), B, N, dm, H, vid, stream))
        else:
            _lib.check(lib.qmha_solve_ws(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), B, N, dm, H, vid,
                                         ws.data_ptr(), ws.numel(), stream))
        return O

    nbytes = lib.qmha_workspace_size(B, N, dm, H, vid)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    pg = torch.Generator(device=dev).manual_seed(7)

    def poison():
        ws.random_(0, 256, generator=pg)

    prev = set_fused(0)
    pw = lib.qmha_debug_set_int8_fused_wait(5000)
    failures = []

    def expect(tag, out, i):
        torch.cuda.synchronize()
        if not torch.equal(out, refs[i]):
            failures.append(f"{tag}: set {i}, max |diff| {(out - refs[i]).abs().nan_to_num(1e30).max().item():.3g}")

    try:
        refs = [call(i) for i in range(3)]  # two launches, library workspace (left holding X2's bytes)
        torch.cuda.synchronize()
        for r in refs:
            assert torch.isfinite(r).all()
        set_fused(1)
        for i in range(3):  # 1
            poison()
            expect("poisoned", call(i, ws), i)
        for i in (0, 1, 2, 0):  # 2
            expect("back-to-back", call(i, ws), i)
        for i in (0, 1):  # 3
            expect("library workspace", call(i), i)
        if is8:
            lib.qmha_debug_set_int8_fused_wait(0)  # 4
            poison()
            expect("forced self-production", call(1, ws), 1)
            lib.qmha_debug_set_int8_fused_wait(5000)
        set_fused(2)  # 5
        for i in (1, 2):
            poison()
            expect("cross-XCD rule", call(i, ws), i)
    finally:
        set_fused(prev)
        lib.qmha_debug_set_int8_fused_wait(pw)
    assert pw == 5000
    assert not failures, "; ".join(failures)


def test_int8_default_call_is_fused_and_equals_two_launch(dev):
    """The library's default per-block call (mode as shipped) equals the two-launch call bit for bit at the C4
    shape on fresh inputs, with the library workspace holding another input set's bytes."""
    from quantizedmha_amd import _lib
    lib = _lib.load()
    vid = _lib.variant_id("fa_tc_int8_b")
    B, N, H, d = 16, 4096, 16, 64
    stream = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev).manual_seed(99)
    X = [tuple(torch.randn(B, N, H * d, device=dev, generator=g) for _ in range(3)) for _ in range(2)]

    def call(i):
        Q, K, V = X[i]
        O = torch.empty_like(Q)
        _lib.check(lib.qmha_solve_ex(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), B, N, H * d, H, vid, stream))
        return O

    shipped = lib.qmha_debug_set_int8_fused(0)
    lib.qmha_debug_set_int8_fused(shipped)
    prev = lib.qmha_debug_set_int8_fused(0)
    try:
        ref0 = call(0)
        ref1 = call(1)
        lib.qmha_debug_set_int8_fused(shipped)
        out0 = call(0)  # the workspace holds X1's bytes
        torch.cuda.synchronize()
    finally:
        lib.qmha_debug_set_int8_fused(prev)
    assert torch.equal(out0, ref0)
    assert not torch.equal(ref0, ref1)


@pytest.mark.parametrize("variant,B,N,H,d", [("fa_tc_int8_b", 2, 1024, 8, 64), ("fa_tc_int8_b", 1, 512, 4, 32),
                                             ("fa_tc_int8_b", 2, 512, 2, 128), ("fa_tc_v1a", 2, 1024, 8, 64)])
def test_fused_nan_inf_groups_bit_identical(dev, variant, B, N, H, d):
    """The fused producer's fast quantiser detects a NaN or an infinity in a K / V group from its magic-biased
    results and redoes that group exactly (NaN -> 0, an infinity makes the group scale inf and every value 0,
    as the reference's fp32_to_int8sram).  Groups with NaN / +-inf in K and V, one group all-NaN: the fused call
    equals the two-launch call bit for bit, on a poisoned caller workspace.  The fp16 form converts NaN / inf
    as the pre-pass does (RNE), so its NaNs propagate identically."""
    from quantizedmha_amd import _lib
    lib = _lib.load()
    vid = _lib.variant_id(variant)
    set_fused = lib.qmha_debug_set_int8_fused if variant == "fa_tc_int8_b" else lib.qmha_debug_set_f16_fused
    dm = H * d
    stream = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev).manual_seed(5)
    Q, K, V = (torch.randn(B, N, dm, device=dev, generator=g) for _ in range(3))
    K[0, 3, 5] = float("nan")
    K[0, 40, (2 * d + 1) % dm] = float("inf")
    K.view(torch.int32)[0, 300, 3] = 0x7F800001  # a signalling NaN with a payload
    V.view(torch.int32)[0, 301, 2] = -0x3FFFFF  # a negative quiet NaN with a payload (0xFFC00001)
    V[0, 70, 7] = float("nan")
    V[-1, 100, d + 3] = float("-inf")
    V[-1, 128:160, 0:d] = float("nan")  # a whole group
    K[0, 200, 1] = -float("inf")
    nbytes = lib.qmha_workspace_size(B, N, dm, H, vid)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)

    def call(fused):
        O = torch.empty_like(Q)
        prev = set_fused(fused)
        try:
            ws.random_(0, 256)
            _lib.check(lib.qmha_solve_ws(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), B, N, dm, H, vid,
                                         ws.data_ptr(), ws.numel(), stream))
            torch.cuda.synchronize()
        finally:
            set_fused(prev)
        return O

    ref, out = call(0), call(1)
    assert torch.equal(torch.nan_to_num(ref, 7.0), torch.nan_to_num(out, 7.0))
