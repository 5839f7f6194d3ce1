"""Re-entrancy of the drop-in boundary (the reference's `solve` is re-entrant in practice --
per-call cudaMalloc'd scratch and private streams, include/launchers.h:27-33,64-71).

The library caches its scratch per (device, stream) instead, and a call holds a lease on that slot from the
moment the buffer is handed out until its last kernel is enqueued (qmha_api.cpp, lease_workspace).  These
tests run concurrent host threads through every C-ABI entry a binding uses -- the per-variant `solve` of
libqmha_fa_tc_int8_b.so (blocking, null stream), qmha_solve_ex on one SHARED stream, and the ctypes
jax_ext.flash_solve (blocking, which releases the GIL like the torch ctypes front-end) -- with different
inputs and growing problem sizes (so the slot's buffer is retired and reallocated while other threads'
work is in flight), and require every output to be bit-identical to the same call made single-threaded.

And the scratch contents never matter: qmha_solve_ws on a caller workspace full of random bytes, or left
holding another input set's intermediates, gives the library call's output bit for bit."""
import ctypes
import os
import threading

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from quantizedmha_amd import _lib
    _lib.load()  # raises if the HIP library is missing: no silent fallback
    return torch.device("cuda:0")


THREADS, CALLS = 4, 25
H, D = 4, 64
VARIANTS = ("fa_tc_int8_b", "fa_tc_int8_pt", "fa_tc_v1a")
ENTRIES = ("solve", "solve_ex", "jax")


def _plan(t, j):
    """(entry, variant, B, N) of call j of thread t: every entry point and variant in every thread, and N
    growing over the run (the largest size of each thread first appears at call >= 9, so its slot grows
    while the other threads' work is in flight)."""
    entry = ENTRIES[(j + t) % 3]
    variant = "fa_tc_int8_b" if entry == "solve" else VARIANTS[(j + 2 * t) % 3]
    B = 2 if entry == "solve_ex" else 1
    N = (128, 256, 96, 512, 160, 1024, 384)[min(j // 3, 6) if j % 4 else (j + t) % 4]
    return entry, variant, B, N


def test_concurrent_callers_bit_identical(dev):
    from quantizedmha_amd import _lib, jax_ext
    lib = _lib.load()
    solve_lib = ctypes.CDLL(os.path.join(ROOT, "quantizedmha_amd", "lib", "libqmha_fa_tc_int8_b.so"))
    solve_lib.solve.restype = None
    solve_lib.solve.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3
    shared = torch.cuda.Stream(dev)
    sptr = shared.cuda_stream
    calls = {}
    for t in range(THREADS):
        for j in range(CALLS):
            entry, variant, B, N = _plan(t, j)
            g = torch.Generator(device=dev).manual_seed(1000 * t + j)
            Q, K, V = (torch.randn(B, N, H * D, device=dev, generator=g) * (0.4 + 0.05 * j) for _ in range(3))
            calls[t, j] = (entry, variant, B, N, Q, K, V, torch.full_like(Q, float("nan")))
    # single-threaded references: the same variant on the same inputs, one call at a time
    refs = {}
    for key, (entry, variant, B, N, Q, K, V, _) in calls.items():
        R = torch.empty_like(Q)
        _lib.check(lib.qmha_solve_ex(Q.data_ptr(), K.data_ptr(), V.data_ptr(), R.data_ptr(), B, N, H * D, H,
                                     _lib.variant_id(variant), None))
        torch.cuda.synchronize(dev)
        refs[key] = R
    lib.qmha_release_workspaces()  # every slot starts empty: the threads' calls grow them
    torch.cuda.synchronize(dev)
    errors = []
    start = threading.Barrier(THREADS)

    def worker(t):
        try:
            torch.cuda.set_device(dev)
            start.wait()
            for j in range(CALLS):
                entry, variant, B, N, Q, K, V, O = calls[t, j]
                if entry == "solve":  # blocking, null stream (reference launchers.h:64)
                    solve_lib.solve(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), N, H * D, H)
                elif entry == "solve_ex":  # asynchronous, one stream shared by all threads
                    _lib.check(lib.qmha_solve_ex(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), B, N, H * D,
                                                 H, _lib.variant_id(variant), sptr))
                else:  # the ctypes raw-pointer binding (extensions/jax/jax_ext.cpp), blocking
                    jax_ext.flash_solve(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), N, H * D, H, variant)
        except Exception as e:  # reported below; the other threads go on
            errors.append(f"thread {t}: {e!r}")

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(THREADS)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=90)
    assert not any(th.is_alive() for th in threads), "a caller thread hung"
    shared.synchronize()
    torch.cuda.synchronize(dev)
    assert not errors, errors
    bad = []
    for key, (entry, variant, B, N, Q, K, V, O) in calls.items():
        if not torch.equal(O, refs[key]):
            d = (O - refs[key]).abs().nan_to_num(1e30).max().item()
            bad.append(f"thread {key[0]} call {key[1]} {entry} {variant} B{B} N{N}: max|diff| {d:.3g}")
    assert not bad, f"{len(bad)} of {len(calls)} calls differ from their single-threaded result: " + "; ".join(bad[:8])
    seen = {(c[0], c[1]) for c in calls.values()}
    assert {e for e, _ in seen} == set(ENTRIES) and {v for _, v in seen} == set(VARIANTS), seen


@pytest.mark.parametrize("variant,B,N,d", [("fa_tc_int8_b", 3, 1024, 64), ("fa_tc_int8_b", 2, 96, 32),
                                           ("fa_tc_int8_pt", 3, 1024, 64), ("fa_tc_int8_pt", 2, 512, 128),
                                           ("fa_tc_v1a", 3, 1024, 64), ("fa_tc_int8_b", 1, 256, 96)])
def test_scratch_contents_never_matter(dev, variant, B, N, d):
    """qmha_solve_ws on a caller workspace of random bytes, then back-to-back calls of three input sets on it
    without refilling (each call's scratch holds the previous set's intermediates): every output equals the
    library call's bit for bit."""
    from quantizedmha_amd import _lib
    lib = _lib.load()
    vid = _lib.variant_id(variant)
    Hh = 4
    dm = Hh * d
    stream = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev).manual_seed(31 + N + B + d)
    sets = [tuple(torch.randn(B, N, dm, device=dev, generator=g) * (0.5 + 0.25 * i) for _ in range(3)) for i in range(3)]

    def call(i, ws=None):
        Q, K, V = sets[i]
        O = torch.full_like(Q, float("nan"))
        if ws is None:
            _lib.check(lib.qmha_solve_ex(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), B, N, dm, Hh, vid, stream))
        else:
            _lib.check(lib.qmha_solve_ws(Q.data_ptr(), K.data_ptr(), V.data_ptr(), O.data_ptr(), B, N, dm, Hh, vid,
                                         ws.data_ptr(), ws.numel(), stream))
        torch.cuda.synchronize(dev)
        return O

    refs = [call(i) for i in range(3)]
    for r in refs:
        assert torch.isfinite(r).all()
    ws = torch.empty(lib.qmha_workspace_size(B, N, dm, Hh, vid), dtype=torch.uint8, device=dev)
    for i in range(3):
        ws.random_(0, 256)
        assert torch.equal(call(i, ws), refs[i]), f"poisoned workspace, set {i}"
    for i in (2, 0, 1, 2):
        assert torch.equal(call(i, ws), refs[i]), f"back-to-back, set {i}"
    assert not torch.equal(refs[0], refs[1])
