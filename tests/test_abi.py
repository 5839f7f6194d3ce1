"""CPU tests of the drop-in boundary: the C-ABI libraries load and export every symbol
include/launchers.h declares, host-side argument checks reject bad shapes before any GPU
call, and the Python mirrors of the reference bindings keep its error behaviour.
No kernel is launched here (no GPU in the build container)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "launchers.h")
LIB_DIR = os.path.join(ROOT, "quantizedmha_amd", "lib")
VARIANTS = ["fa", "fa_tc_v1a", "fa_tc_int8_b", "unfused", "fa_mfma", "fa_tc_int8_pt"]


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*([a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


@pytest.fixture(scope="module")
def built():
    from tools.build import build
    build(verbose=False)
    return True


def test_header_declares_reference_solve_signature():
    src = open(HEADER).read()
    assert re.search(r"void solve\(const float \*Q, const float \*K, const float \*V, float \*output, int N, "
                     r"int d_model, int h\);", src)


def test_libqmha_exports_every_declared_symbol(built):
    lib = ctypes.CDLL(os.path.join(LIB_DIR, "libqmha.so"))
    names = declared_functions()
    assert "solve" in names and "qmha_solve_ex" in names and len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n


@pytest.mark.parametrize("variant", VARIANTS)
def test_variant_libraries_export_solve(built, variant):
    path = os.path.join(LIB_DIR, f"libqmha_{variant}.so")
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    assert re.search(r" T solve$", out, flags=re.M), out
    ctypes.CDLL(path)  # resolves libqmha.so through $ORIGIN


def test_python_binding_signatures_cover_header(built):
    from quantizedmha_amd import _lib
    assert set(declared_functions()) == set(_lib.SIGNATURES)
    lib = _lib.load()
    assert lib.qmha_version().decode().startswith("qmha-mi355x")


def test_host_side_queries(built):
    from quantizedmha_amd import _lib
    lib = _lib.load()
    for name, vid in _lib.VARIANTS.items():
        assert lib.qmha_variant_from_name(name.encode()) == vid
        assert lib.qmha_variant_name(vid).decode() == name
    assert lib.qmha_variant_from_name(b"fa_tc_v2") == -1
    # int8 workspace: int8 K, V as f16-valued integers (main-kernel operand), the K and V scales --
    # no Q: the main kernel quantises Q in registers (round-2 VERDICT: 67 MB of dead Qi / sQ at C4)
    ws = lib.qmha_workspace_size(16, 4096, 1024, 16, 2)
    assert ws >= 3 * 16 * 16 * 4096 * 64 and ws < 3 * 16 * 16 * 4096 * 64 * 1.01
    assert lib.qmha_workspace_size(2, 256, 128, 2, 0) == 0  # scalar path needs no scratch
    assert lib.qmha_status_string(1).decode() == "invalid argument"


@pytest.mark.parametrize("args,err", [
    ((1, 100, 128, 2, 2), "N must be a multiple of 32"),
    ((1, 128, 130, 2, 2), "head size"),
    ((1, 128, 96, 2, 2), "multiple of 32"),   # d = 48 (config.h:32)
    ((1, 128, 1024, 2, 2), "above 256"),      # d = 512
    ((1, 128, 192, 2, 5), "d = 32, 64, 128"),  # d = 96 in the per-tensor mode
    ((1, 128, 128, 3, 2), "divisible"),
    ((1, 128, 128, 2, 7), "unknown variant"),
    ((0, 128, 128, 2, 2), "positive"),
])
def test_invalid_shapes_rejected_before_launch(built, args, err):
    from quantizedmha_amd import _lib
    lib = _lib.load()
    dummy = ctypes.c_void_p(0x1000)  # never dereferenced: checks run first
    B, N, dm, h, v = args
    st = lib.qmha_solve_ex(dummy, dummy, dummy, dummy, B, N, dm, h, v, None)
    assert st in (1, 4)
    assert err in lib.qmha_last_error().decode()
    st = lib.qmha_solve_ex(None, dummy, dummy, dummy, 1, 128, 128, 2, 2, None)
    assert st == 1 and "null" in lib.qmha_last_error().decode()


def test_torch_binding_error_behaviour_matches_reference():
    torch = pytest.importorskip("torch")
    from quantizedmha_amd import torch_ext
    q = torch.zeros(64, 32)
    with pytest.raises(RuntimeError, match="Inputs must be CUDA tensors"):  # torch_ext.cpp:14
        torch_ext.flash_solve(q, q, q, 32, 4)
    with pytest.raises(RuntimeError, match="Inputs must be CUDA tensors"):
        torch_ext.flash_solve(q.double(), q, q, 32, 4)


def test_torch_mirror_shape_rules():
    """[B, N, d_model] is B sequences; any other shape is one sequence of numel/d_model rows (the
    reference's rule, torch_ext.cpp:23-25); round-2 ADVICE: [32, 64, 32] with d_model = 1024 used
    to launch B = 32, N = 64 over a 65,536-float buffer."""
    torch = pytest.importorskip("torch")
    from quantizedmha_amd import torch_ext
    assert torch_ext._shape(torch.zeros(32, 64, 32), 1024) == (1, 64)
    assert torch_ext._shape(torch.zeros(2, 128, 256), 256) == (2, 128)
    assert torch_ext._shape(torch.zeros(128, 4, 64), 256) == (1, 128)
    assert torch_ext._shape(torch.zeros(96, 256), 256) == (1, 96)
    with pytest.raises(RuntimeError, match="divisible by d_model"):
        torch_ext._shape(torch.zeros(10, 10), 64)


def test_jax_binding_imports_without_jax():
    from quantizedmha_amd import jax_binding, jax_ext  # noqa: F401
    try:
        import jax  # noqa: F401
    except ImportError:
        with pytest.raises(ImportError):
            jax_binding.flash_solve_jax(None, None, None, 32, 4)


def test_driver_help_runs_without_gpu(built):
    exe = os.path.join(ROOT, "quantizedmha_amd", "bin", "qmha_profile")
    r = subprocess.run([exe, "--help"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0
    assert "fa_tc_int8_b" in r.stdout and "--warmup" in r.stdout


def test_slot_permutations_are_bijective():
    """Python restatement of qmha_common.hpp's operand slot maps: each is a permutation of
    0..31 and matches the MFMA accumulator row map used for P^T."""
    acc_row = lambda r, h: (r & 3) + 8 * (r >> 2) + 4 * h  # noqa: E731
    kv_i8 = [acc_row(s & 15, s >> 4) for s in range(32)]
    assert sorted(kv_i8) == list(range(32))
    slot_i8 = lambda kv: 16 * ((kv >> 2) & 1) + 4 * (kv >> 3) + (kv & 3)  # noqa: E731
    assert all(slot_i8(kv_i8[s]) == s for s in range(32))
    kv_f16 = [16 * (s >> 4) + 4 * ((s >> 3) & 1) + (s & 3) + 8 * ((s >> 2) & 1) for s in range(32)]
    assert sorted(kv_f16) == list(range(32))
    # f16 k-step s takes accumulator registers 8s..8s+7 of lane half h
    for s in range(2):
        for h in range(2):
            for e in range(8):
                assert kv_f16[16 * s + 8 * h + e] == acc_row(8 * s + e, h)
    assert np.array_equal(np.argsort(kv_f16), [16 * (kv >> 4) + 8 * ((kv >> 2) & 1) + (kv & 3) + 4 * ((kv >> 3) & 1)
                                               for kv in range(32)])


def test_production_library_has_one_kernel_per_variant_and_d(built):
    """No tuning/ablation alternates in the shipped libqmha.so (round-1 ADVICE): every kernel
    template is instantiated at most once per head size, and no QMHA_*_CFG / overlap
    environment switch exists (those live in QMHA_ABLATION builds only)."""
    path = os.path.join(LIB_DIR, "libqmha.so")
    syms = subprocess.run(["nm", path], capture_output=True, text=True, check=True).stdout
    stubs = set(re.findall(r"__device_stub__(\w+?)ILi(\d+)E(\w*)", syms))
    per = {}
    dumps = []
    for name, d, rest in stubs:
        if name.startswith("qmha_gemm"):
            continue
        if name == "qmha_fa_int8_pt_v3_kernel":  # <D, WAVES, SG, DUMP> (per-tensor, d = 64)
            if "Lb1E" in rest:
                dumps.append((name, d, rest.replace("Lb1E", "Lb0E", 1)))
                continue
            per.setdefault((name, d), set()).add(rest)
            continue
        if name == "qmha_fa_int8_pipe_kernel":  # <D, WAVES, FL>
            m, fl = re.match(r"Li(\d+)ELi(\d+)E", rest), 2
        elif name == "qmha_fa_int8_kernel":  # <D, FL> (the one-tile kernel: N = 32, and d outside 32/64/128)
            m, fl = re.match(r"Li(\d+)E", rest), 1
        else:
            m = None
        if m and int(m.group(fl)) & 1048576:  # FL_PT: the fa_tc_int8_pt variant's own instance
            name += "[pt]"
        if m and int(m.group(fl)) & 256:  # FL_DUMP: the test-hook twin of the production instance
            f = m.group(fl)
            twin = rest.replace(f"Li{f}E", f"Li{int(f) & ~256}E", 1) if fl == 1 else \
                rest.replace(f"ELi{f}E", f"ELi{int(f) & ~256}E", 1)
            dumps.append((name, d, twin))
            continue
        per.setdefault((name, d), set()).add(rest)
    # per-block d = 32 / 64 / 128 (pipelined) and 96 / 160 / 192 / 224 / 256 (one-tile kernel),
    # per-tensor d = 32 / 64 / 128
    assert len(dumps) == 11, dumps
    for name, d, twin in dumps:  # exactly the production schedule (same WAVES, flags, PAD) plus the stores
        if name == "qmha_fa_int8_pt_v3_kernel":  # the 8-wave production instance (the 4-wave one has no twin)
            assert twin in per[(name, d)], (name, d, twin)
        else:
            assert per[(name, d)] == {twin}, (name, d, twin)
    assert per, syms[:2000]
    for (name, d), inst in per.items():
        # the V layout and the per-tensor mode are template arguments of the quantiser; the any-d
        # pre-pass is instantiated for the int8 V layouts and the fp16 conversion
        limit = 3 if name in ("qmha_quant_int8_kernel", "qmha_prepass_any_kernel") else 1
        if name == "qmha_fa_int8_pt_v3_kernel":  # 8-wave workgroups, 4-wave ones for one-CU-each grids
            limit = 2
        assert len(inst) <= limit, (name, d, sorted(inst))
    blob = open(path, "rb").read()
    for env in (b"QMHA_INT8_CFG", b"QMHA_F16_CFG", b"QMHA_F32_CFG", b"QMHA_OVERLAP_CHUNKS", b"QMHA_INT8_ABL"):
        assert env not in blob, env


def test_fa_scalar_kernel_has_no_matrix_core_instructions(built):
    """BASELINE C2 as written ("fa (no tensor cores) ... scalar HIP, LDS tiling only"): the
    shipped fa kernel (qmha_fa_f32_v3_kernel) contains no v_mfma instruction; its fa_mfma
    sibling (qmha_fa_f32_mfma_kernel) does."""
    from tools.isa import disasm
    asm, _ = disasm(os.path.join(ROOT, "build", "obj", "qmha_fa_f32.o"))  # the object linked into libqmha.so
    funcs = {f.split("\n", 1)[0]: f for f in re.split(r"\n(?=[0-9a-f]+ <)", asm)}
    scalar = [k for k in funcs if "qmha_fa_f32_v3_kernel" in k]
    mfma = [k for k in funcs if "qmha_fa_f32_mfma_kernel" in k]
    assert len(scalar) == 8 and len(mfma) == 8, (scalar, mfma)  # d = 32, 64, ..., 256
    for k in scalar:
        assert "v_mfma" not in funcs[k] and "v_fma_f32" in funcs[k], k
    for k in mfma:
        assert "v_mfma_f32_32x32x2" in funcs[k], k


def test_compiled_torch_ext_imports_with_reference_signature(built):
    """The compiled `torch_ext` module (reference extensions/torch/torch_ext.cpp:45-57) imports
    by its reference name, keeps the argument names/defaults and rejects non-GPU inputs with
    the reference message before touching the device."""
    import sys
    import torch
    sys.path.insert(0, LIB_DIR)
    try:
        import torch_ext
    finally:
        sys.path.pop(0)
    doc = torch_ext.flash_solve.__doc__
    assert "flash_solve(Q: torch.Tensor, K: torch.Tensor, V: torch.Tensor, d_model" in doc
    assert "kernel: str = 'fa_tc_int8_b'" in doc
    x = torch.zeros(64, 64)
    with pytest.raises(RuntimeError, match="Inputs must be CUDA tensors"):
        torch_ext.flash_solve(x, x, x, 64, 1)


def test_lds_swizzle16_conflict_free():
    """qmha_common.hpp kswz16 / vswz16 restated: every ds_read_b128 lane group of the 16x16 kernels'
    K and V^T operand reads (MI355X_MICROARCH.md §LDS: 4 groups of 16 lanes, bank (a/4) mod 64) hits 16
    distinct 16-byte slots of the 256-byte bank row, and each mask is an XOR (a bijection per row)."""
    groups = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
              list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
    groups += [[lane + 32 for lane in g] for g in groups]
    kap16 = lambda kb, m: 16 * (m >> 3) + 4 * ((m >> 2) & 1) + (m & 3) + 8 * kb  # noqa: E731
    kswz = {64: lambda r: 2 * ((r >> 4) & 1),
            128: lambda r: ((r >> 1) & 1) ^ (2 * ((r >> 2) & 1)) ^ (4 * ((r >> 4) & 1)),
            256: lambda r: (r & 1) ^ (2 * ((r >> 1) & 1)) ^ (4 * ((r >> 2) & 1)) ^ (8 * ((r >> 4) & 1))}
    vswz = lambda d: (2 * ((d >> 2) & 1)) ^ (3 * ((d >> 3) & 1))  # noqa: E731
    for rb, f in kswz.items():  # K rows: int8 d = rb, f16 d = rb / 2
        assert all(f(r) < rb // 16 for r in range(64))
        for gi in range(2):
            for kb in range(2):
                for ks in range(rb // 64):
                    for g in groups:
                        slots = []
                        for lane in g:
                            row = 32 * gi + kap16(kb, lane & 15)
                            slots.append((row * rb // 16 + ((4 * ks + (lane >> 4)) ^ f(row))) % 16)
                        assert len(set(slots)) == 16, (rb, gi, kb, ks)
    for m in range(8):  # V^T rows d = 16 m + r16, chunk = lane group
        for g in groups:
            slots = [(4 * ((16 * m + (lane & 15)) & 3) + ((lane >> 4) ^ vswz(16 * m + (lane & 15)))) % 16 for lane in g]
            assert len(set(slots)) == 16, m
