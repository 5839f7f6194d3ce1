"""JAX helper: mirror of the reference's extensions/jax/jax_binding.py (flash_solve_jax).

The reference converts JAX -> DLPack -> CuPy to get device pointers and back
(jax_binding.py:25-77).  CuPy is not part of this stack; the MI355X build uses
torch.from_dlpack (PyTorch-ROCm) for the same zero-copy pointer hand-off, then calls
jax_ext.flash_solve.  JAX is imported lazily: it is not installed in the build image, so
this module imports fine and flash_solve_jax raises ImportError only when called.
"""
from __future__ import annotations

from . import _lib, jax_ext


def flash_solve_jax(q, k, v, d_model, num_heads, kernel: str = _lib.DEFAULT_KERNEL):
    import jax.dlpack as jdlpack  # noqa: F401  (ImportError if JAX is absent)
    import torch

    def to_torch(a):
        t = torch.from_dlpack(a)
        return t.to(torch.float32).contiguous()

    qt, kt, vt = to_torch(q), to_torch(k), to_torch(v)
    out = torch.empty_like(qt)
    torch.cuda.synchronize(qt.device)
    jax_ext.flash_solve(qt.data_ptr(), kt.data_ptr(), vt.data_ptr(), out.data_ptr(), int(qt.shape[0]),
                        int(d_model), int(num_heads), kernel)
    return jdlpack.from_dlpack(out)
