"""Raw-pointer binding: mirror of the reference's extensions/jax/jax_ext.cpp (jax_ext.flash_solve).

flash_solve(q_ptr, k_ptr, v_ptr, out_ptr, N, d_model, num_heads, kernel='fa_tc_int8_b') -> None
Device pointers are integer addresses of fp32 [N, d_model] buffers.  Like the reference's
`solve`, the call is blocking.  Unlike the reference (which ignored `kernel`, :19), the
named variant is used; errors raise instead of being ignored.
"""
from __future__ import annotations

import ctypes

from . import _lib


def flash_solve(q_ptr: int, k_ptr: int, v_ptr: int, out_ptr: int, N: int, d_model: int, num_heads: int,
                kernel: str = _lib.DEFAULT_KERNEL) -> None:
    vid = _lib.VARIANTS.get(kernel, _lib.VARIANTS[_lib.DEFAULT_KERNEL])
    st = _lib.load().qmha_solve_variant(ctypes.c_void_p(q_ptr), ctypes.c_void_p(k_ptr), ctypes.c_void_p(v_ptr),
                                        ctypes.c_void_p(out_ptr), int(N), int(d_model), int(num_heads), vid)
    _lib.check(st, f"jax_ext.flash_solve({kernel})")
