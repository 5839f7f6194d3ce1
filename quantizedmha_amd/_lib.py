"""ctypes binding of the native C-ABI (include/launchers.h) -- the only way the Python
layer reaches the HIP kernels.  There is no fallback: if libqmha.so is missing or fails to
load, every entry point raises, so a GPU run can never silently take another path."""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(HERE, "lib")
# QMHA_LIB_PATH: load another build of the same C-ABI (A/B kernel experiments); still no fallback
LIB_PATH = os.environ.get("QMHA_LIB_PATH") or os.path.join(LIB_DIR, "libqmha.so")

VARIANTS = {"fa": 0, "fa_tc_v1a": 1, "fa_tc_int8_b": 2, "unfused": 3, "fa_mfma": 4, "fa_tc_int8_pt": 5}
DEFAULT_KERNEL = "fa_tc_int8_b"
QMHA_OK = 0

# every symbol include/launchers.h declares, with its ctypes signature
_i, _sz, _vp, _cp = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_char_p
SIGNATURES = {
    "solve": (None, [_vp, _vp, _vp, _vp, _i, _i, _i]),
    "qmha_solve_ex": (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "qmha_workspace_size": (_sz, [_i, _i, _i, _i, _i]),
    "qmha_solve_ws": (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _vp, _sz, _vp]),
    "qmha_solve_variant": (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _i]),
    "qmha_quantize_int8": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _i, _vp]),
    "qmha_debug_qk_int32": (_i, [_vp, _vp, _i, _i, _i, _i, _vp]),
    "qmha_debug_fa_int8_dump": (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp]),
    "qmha_debug_fa_int8_pt_dump": (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp]),
    "qmha_variant_from_name": (_i, [_cp]),
    "qmha_variant_name": (_cp, [_i]),
    "qmha_status_string": (_cp, [_i]),
    "qmha_version": (_cp, []),
    "qmha_last_error": (_cp, []),
    "qmha_profile_enable": (None, [_i]),
    "qmha_set_overlap_chunks": (_i, [_i]),
    "qmha_debug_set_pt_wait": (ctypes.c_longlong, [ctypes.c_longlong]),
    "qmha_profile_collect": (_i, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong),
                                  ctypes.POINTER(ctypes.c_double)]),
    "qmha_release_workspaces": (None, []),
}

_lock = threading.Lock()
_lib = None


class QMHAError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load libqmha.so (built by tools/build.py / __graft_entry__.build())."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise QMHAError(f"native library {path} not found: run `python tools/build.py` "
                                "(quantizedmha_amd has no non-HIP fallback)")
            lib = ctypes.CDLL(path)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def check(status: int, what: str = "qmha") -> None:
    if status != QMHA_OK:
        lib = load()
        raise QMHAError(f"{what}: {lib.qmha_status_string(status).decode()}: {lib.qmha_last_error().decode()}")


def variant_id(kernel: str) -> int:
    if kernel not in VARIANTS:
        raise KeyError(kernel)
    return VARIANTS[kernel]
