"""quantizedmha_amd -- MI355X (gfx950) native fused multi-head attention forward.

Drop-in for MattJBorowski1991/QuantizedMHA's `solve` path (include/launchers.h) and its
extension entry points:
  * torch_ext.flash_solve(Q, K, V, d_model, num_heads, kernel='fa_tc_int8_b')
      (reference extensions/torch/torch_ext.cpp:11-57)
  * jax_ext.flash_solve(q_ptr, k_ptr, v_ptr, out_ptr, N, d_model, num_heads, kernel)
      (reference extensions/jax/jax_ext.cpp:12-37)
  * jax_binding.flash_solve_jax(q, k, v, d_model, num_heads, kernel)
      (reference extensions/jax/jax_binding.py:25-77)
All of them call the C-ABI in quantizedmha_amd/lib/libqmha.so (hand-written HIP kernels).
"""
from ._lib import DEFAULT_KERNEL, VARIANTS, QMHAError, load  # noqa: F401

__all__ = ["DEFAULT_KERNEL", "VARIANTS", "QMHAError", "load"]
__version__ = "0.1.0"
