"""The fused per-block int8 call (FL_FUSED), an opt-in (qmha_debug_set_int8_fused(1);
the library's default is the two-launch path): bit-identity with the default path.  In a file of its own
that sorts after every other GPU test file, so that a failure of the opt-in path cannot stop the rest of
a `pytest -x -m gpu` run."""
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


@pytest.mark.parametrize("B,N,H,d", [(2, 1024, 8, 64), (4, 4096, 16, 64), (1, 8192, 32, 32), (2, 512, 8, 32),
                                     (2, 2048, 4, 128), (3, 96, 2, 64), (5, 2080, 3, 64), (1, 65536, 1, 64)])
def test_int8_fused_bit_identical(dev, B, N, H, d):
    """With the opt-in, the per-block call at d = 32 / 64 / 128 is one kernel that quantises K / V itself (FL_FUSED,
    DESIGN.md 5.2d): workgroups produce K / V groups for each other under agent-coherent stores and
    per-group flags.  Its output must equal the two-launch path (pre-pass, then the same sweep) bit for
    bit -- with the default work split, with every wave producing its own head after a zero wait
    bound, and (one round, grid % 8 == 0) with every group produced by a workgroup of another XCD.
    Shapes: C4-like, the reference's (2 rounds at d = 32), d = 128, N = 96 (nqb = 1), a ragged grid
    whose heads straddle the XCD ranges and rounds (B5 H3 N2080), and one head longer than a round
    (N = 65536: the launcher routes it to the two launches, tests/test_fused_schedule.py)."""
    from quantizedmha_amd import _lib, torch_ext
    lib = _lib.load()
    g = torch.Generator(device=dev).manual_seed(31)
    Q, K, V = (torch.randn(B, N, H * d, device=dev, generator=g) * 0.5 for _ in range(3))
    ref = torch_ext.flash_solve(Q, K, V, H * d, H, kernel="fa_tc_int8_b")  # the default: two launches
    torch.cuda.synchronize()
    prev = lib.qmha_debug_set_int8_fused(1)
    try:
        out = torch_ext.flash_solve(Q, K, V, H * d, H, kernel="fa_tc_int8_b")
        torch.cuda.synchronize()
        pw = lib.qmha_debug_set_int8_fused_wait(0)
        try:
            forced = torch_ext.flash_solve(Q, K, V, H * d, H, kernel="fa_tc_int8_b")
            torch.cuda.synchronize()
        finally:
            lib.qmha_debug_set_int8_fused_wait(pw)
        nwg = B * H * -(-N // 128)
        cross = None
        if nwg % 8 == 0 and nwg <= 512:
            lib.qmha_debug_set_int8_fused(2)
            cross = torch_ext.flash_solve(Q, K, V, H * d, H, kernel="fa_tc_int8_b")
            torch.cuda.synchronize()
    finally:
        lib.qmha_debug_set_int8_fused(prev)
    assert prev == 0 and pw == 5000
    assert torch.equal(out, ref), (out - ref).abs().max().item()
    assert torch.equal(forced, ref)
    if cross is not None:
        assert torch.equal(cross, ref)
