#!/usr/bin/env python3
"""Build the MI355X (gfx950) native library, per-variant `solve` libraries and the driver.

    python tools/build.py            # incremental
    python tools/build.py --clean

Outputs (in-tree, git-ignored, shipped to the GPU box with the snapshot):
    quantizedmha_amd/lib/libqmha.so                 all C-ABI entry points (include/launchers.h)
    quantizedmha_amd/lib/libqmha_<variant>.so       `solve` bound to one kernel (reference Makefile KERNEL=)
    quantizedmha_amd/lib/libqmha_probe.so           bench.py's in-kernel clock probe (qmha_clock_probe.hip)
    quantizedmha_amd/bin/qmha_profile               HIP C++ host driver (reference drivers/main.cu)
    quantizedmha_amd/lib/torch_ext<EXT_SUFFIX>      compiled pybind module `torch_ext` (reference
                                                    extensions/torch/torch_ext.cpp), linked to libqmha.so
No CUDA, no hipify, no multi-backend dispatch: hipcc --offload-arch=gfx950 only.
"""
import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "quantizedmha_amd", "csrc")
# QMHA_ALT=<name>: an A/B build of libqmha.so alone (own object dir, output in
# quantizedmha_amd/alt_lib/<name>/), leaving the production build untouched
ALT = os.environ.get("QMHA_ALT", "")
OBJ = os.path.join(ROOT, "build", "obj_" + ALT if ALT else "obj")
LIB = os.path.join(ROOT, "quantizedmha_amd", "alt_lib", ALT) if ALT else os.path.join(ROOT, "quantizedmha_amd", "lib")
BIN = os.path.join(ROOT, "quantizedmha_amd", "bin")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

KERNEL_SOURCES = ["qmha_fa_int8.hip", "qmha_fa_f16.hip", "qmha_prepass.hip", "qmha_fa_f32.hip", "qmha_unfused.hip",
                  "qmha_api.cpp"]
# profiling builds (QMHA_EXTRA_FLAGS=-DQMHA_ABLATION) enable the tuning alternatives of the fp16 / fp32 / api
# sources.  The r01-r03 int8 experiment source (ablation perturbations, ring / DMA-split / TSHADOW / ACC1
# schedules, the per-workgroup timeline) was removed in round 5 -- it had fallen behind the production
# workspace layout and entry points; it is in git history up to commit 6d5deec
# (tools/ablation/qmha_fa_int8_ablation.hip).  Int8 ablation builds compile the production source.
VARIANTS = {"fa": 0, "fa_tc_v1a": 1, "fa_tc_int8_b": 2, "unfused": 3, "fa_mfma": 4, "fa_tc_int8_pt": 5}
DRIVER_SOURCES = ["driver/main.cpp", "driver/data.cpp", "driver/verify.cpp"]
HEADERS = ["qmha_common.hpp", "qmha_kernels.hpp", "driver/data.h", "driver/verify.h"]

COMMON_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
                "-Wno-unused-variable", "-Wno-unused-lambda-capture", "-munsafe-fp-atomics",
                "-mllvm", "-amdgpu-mfma-vgpr-form"]
# profiling builds only, e.g. QMHA_EXTRA_FLAGS=-DQMHA_ABLATION (rebuild with --clean)
COMMON_FLAGS += os.environ.get("QMHA_EXTRA_FLAGS", "").split()
if os.environ.get("QMHA_AGPR_FORM"):  # A/B: let MFMA accumulators live in AGPRs
    COMMON_FLAGS = [f for f in COMMON_FLAGS if f not in ("-mllvm", "-amdgpu-mfma-vgpr-form")] + ["-DQMHA_MFMA_AGPR"]


def newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.exists(d) and os.path.getmtime(d) > t for d in deps)


def run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise SystemExit(f"build failed: {cmd[-1]}")
    return r


def header_deps():
    deps = [os.path.join(CSRC, h) for h in HEADERS]
    deps.append(os.path.join(ROOT, "include", "launchers.h"))
    return deps


# per-source flags: the int8 softmax is written as scalar fp32 chains on purpose; SLP-packing
# them into v_pk_* needs register pairs the exp results do not land in (a v_mov per pair)
# -fno-honor-nans: fmaxf on MFMA results and running maxima otherwise gets a canonicalising
# v_max (x, x) in front of it (5 per fp16 tile); the main kernels only.  The pre-passes that read the
# caller's Q/K/V (qmha_prepass.hip) keep default IEEE semantics (round-2 ADVICE)
FILE_FLAGS = {"qmha_fa_int8.hip": ["-fno-slp-vectorize", "-fno-honor-nans"] + os.environ.get("QMHA_INT8_FLAGS", "").split(),
              "qmha_fa_f16.hip": ["-fno-slp-vectorize", "-fno-honor-nans"] + os.environ.get("QMHA_F16_FLAGS", "").split(),
              "qmha_fa_f32.hip": os.environ.get("QMHA_F32_FLAGS", "").split()}


def compile_one(src, extra=()):
    out = os.path.join(OBJ, os.path.basename(src).replace(".hip", ".o").replace(".cpp", ".o"))
    if extra:
        out = out.replace(".o", "_" + "_".join(e.strip("-D").replace("=", "") for e in extra) + ".o")
    full = os.path.join(CSRC, src)
    if newer(out, [full] + header_deps() + [__file__]):
        lang = ["-x", "hip"] if src.endswith(".hip") else []
        run([HIPCC] + COMMON_FLAGS + FILE_FLAGS.get(src, []) + list(extra) + ["-I", os.path.join(ROOT, "include"), "-I", CSRC, "-c"] + lang +
            [full, "-o", out])
    return out


def torch_ext_cmd(out, libqmha):
    """Compile line of the compiled `torch_ext` module (host C++ only: hipcc as the C++ compiler,
    PyTorch's headers and libraries, linked against libqmha.so with an $ORIGIN rpath)."""
    import sysconfig
    import torch
    import torch.utils.cpp_extension as ce
    inc = ce.include_paths(device_type="cuda") + [sysconfig.get_paths()["include"], os.path.join(ROOT, "include")]
    libs = ce.library_paths(device_type="cuda")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return ([HIPCC, "-O2", "-std=c++17", "-fPIC", "-shared", "-DTORCH_EXTENSION_NAME=torch_ext", "-DUSE_ROCM",
             f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-Wno-unused-result", "-Wno-deprecated-declarations"] +
            [f"-I{d}" for d in inc] + [os.path.join(CSRC, "torch_ext.cpp"), "-o", out] + [f"-L{d}" for d in libs] +
            ["-L", LIB, "-lqmha", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-ltorch_hip",
             "-Wl,-rpath,$ORIGIN"] + [f"-Wl,-rpath,{d}" for d in libs])


def build_torch_ext(libqmha):
    import sysconfig
    out = os.path.join(LIB, "torch_ext" + sysconfig.get_config_var("EXT_SUFFIX"))
    if newer(out, [os.path.join(CSRC, "torch_ext.cpp"), libqmha, os.path.join(ROOT, "include", "launchers.h"),
                   __file__]):
        run(torch_ext_cmd(out, libqmha))
    return out


def build(jobs=8, verbose=True):
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(LIB, exist_ok=True)
    os.makedirs(BIN, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, KERNEL_SOURCES))
        shim_objs = {} if ALT else {name: ex.submit(compile_one, "qmha_solve_variant.cpp",
                                                    (f"-DQMHA_SOLVE_VARIANT={vid}", f"-DQMHA_SOLVE_NAME={name}"))
                                    for name, vid in VARIANTS.items()}
        drv_objs = [] if ALT else list(ex.map(compile_one, DRIVER_SOURCES))
        shim_objs = {k: v.result() for k, v in shim_objs.items()}
    libqmha = os.path.join(LIB, "libqmha.so")
    if newer(libqmha, objs):
        run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", libqmha] + objs)
    if ALT:
        if verbose:
            print("built (A/B):", libqmha)
        return libqmha
    for name, o in shim_objs.items():
        out = os.path.join(LIB, f"libqmha_{name}.so")
        if newer(out, [o, libqmha]):
            run([HIPCC, "-shared", "-fPIC", "-o", out, o, "-L", LIB, "-lqmha", "-Wl,-rpath,$ORIGIN"])
    probe = os.path.join(LIB, "libqmha_probe.so")  # bench.py's clock probe (not part of the C-ABI library)
    po = compile_one("qmha_clock_probe.hip")
    if newer(probe, [po]):
        run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", probe, po])
    text = build_torch_ext(libqmha)
    driver = os.path.join(BIN, "qmha_profile")
    if newer(driver, drv_objs + [libqmha]):
        run([HIPCC, "-o", driver] + drv_objs + ["-L", LIB, "-lqmha", "-Wl,-rpath,$ORIGIN/../lib"])
    if verbose:
        print("built:", libqmha, "+", len(shim_objs), "variant libs +", os.path.basename(text), "+", driver)
    return libqmha


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args()
    if a.clean:
        shutil.rmtree(os.path.join(ROOT, "build"), ignore_errors=True)
        shutil.rmtree(LIB, ignore_errors=True)
        shutil.rmtree(BIN, ignore_errors=True)
    build(a.j)


if __name__ == "__main__":
    main()
