"""CPU test: HEAD builds from a clean tree.

`__graft_entry__.build()` runs in a temporary copy of the source tree with no build/,
no lib/ and no bin/, so a broken build script can never again ship binaries the sources
cannot reproduce (round-1 VERDICT, "HEAD does not build").  The copy is sources only;
/root/reference is read in place by oracle/Makefile when it exists.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SKIP_DIRS = {".git", "build", "lib", "bin", "alt_lib", "gpurun_out", "_ref", "__pycache__", ".pytest_cache",
             "profiles", "golden"}


def _ignore(_dir, names):
    return [n for n in names if n in SKIP_DIRS or n.endswith((".so", ".o", ".pyc"))]


@pytest.mark.timeout(600)
def test_graft_entry_build_from_clean_copy(tmp_path):
    dst = tmp_path / "repo"
    shutil.copytree(ROOT, dst, ignore=_ignore)
    r = subprocess.run([sys.executable, "-c", "import __graft_entry__ as g; g.build()"], cwd=dst,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    lib = dst / "quantizedmha_amd" / "lib"
    for name in ("libqmha.so", "libqmha_fa.so", "libqmha_fa_tc_v1a.so", "libqmha_fa_tc_int8_b.so",
                 "libqmha_unfused.so", "libqmha_fa_mfma.so", "libqmha_fa_tc_int8_pt.so"):
        assert (lib / name).is_file(), name
    assert (dst / "quantizedmha_amd" / "bin" / "qmha_profile").is_file()
    assert (dst / "oracle" / "liboracle.so").is_file()


@pytest.mark.timeout(600)
def test_ablation_sources_compile(tmp_path):
    """The profiling build (QMHA_EXTRA_FLAGS=-DQMHA_ABLATION, tools/build.py) compiles: every source with
    QMHA_ABLATION-only branches, compile-only, in parallel (round-4 ADVICE: that build had rotted)."""
    import concurrent.futures as cf
    csrc = os.path.join(ROOT, "quantizedmha_amd", "csrc")
    srcs = [n for n in sorted(os.listdir(csrc)) if n.endswith((".hip", ".cpp"))
            and "QMHA_ABLATION" in open(os.path.join(csrc, n)).read()]
    assert srcs, "no source has a QMHA_ABLATION branch"

    def compile_one(n):
        cmd = ["/opt/rocm/bin/hipcc", "-O1", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-DQMHA_ABLATION",
               "-I", os.path.join(ROOT, "include"), "-I", csrc, "-c", os.path.join(csrc, n), "-o", str(tmp_path / (n + ".o"))]
        return n, subprocess.run(cmd, capture_output=True, text=True, timeout=580)

    with cf.ThreadPoolExecutor(len(srcs)) as ex:
        for n, r in ex.map(compile_one, srcs):
            assert r.returncode == 0, n + ": " + r.stderr[-3000:]
