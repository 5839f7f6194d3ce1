"""PyTorch binding: mirror of the reference's extensions/torch/torch_ext.cpp (torch_ext.flash_solve).

Same name, arguments, return value and error behaviour as the reference:
  flash_solve(Q, K, V, d_model, num_heads, kernel='fa_tc_int8_b') -> Tensor shaped like Q
  * non-GPU inputs        -> RuntimeError("Inputs must be CUDA tensors")       (:14)
  * non-fp32 inputs       -> RuntimeError("Q must be float32") etc.            (:15-17)
  * numel % d_model != 0  -> RuntimeError("Q.numel() must be divisible by d_model")  (:24)
  * unknown kernel name   -> warning, routed to the default fa_tc_int8_b       (:32-34)
Differences (additive): `kernel` really selects the variant (the reference only warned and
used its build-time kernel); a 3-D input [B, N, d_model] is treated as B sequences (the
reference has no batch; any other shape is one sequence of numel/d_model rows, as there); K and V
must have Q's shape; work is enqueued on torch's current stream instead of private
streams + a blocking sync (torch orders it with surrounding ops on that stream).
ROCm tensors report device type 'cuda', exactly as the reference's is_cuda() check expects.
"""
from __future__ import annotations

import warnings
from typing import Optional

import torch

from . import _lib


def _shape(Q: torch.Tensor, d_model: int):
    """(B, N): [B, N, d_model] is B sequences; any other layout is one sequence of
    numel / d_model rows, as in the reference (torch_ext.cpp:23-25), e.g. [N, h, d]."""
    n = Q.numel()
    if d_model <= 0 or n % d_model != 0:
        raise RuntimeError("Q.numel() must be divisible by d_model")
    if Q.dim() == 3 and Q.shape[2] == d_model:
        return Q.shape[0], Q.shape[1]
    return 1, n // d_model


def flash_solve(Q: torch.Tensor, K: torch.Tensor, V: torch.Tensor, d_model: int, num_heads: int,
                kernel: str = _lib.DEFAULT_KERNEL, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """FlashAttention solve (HIP).  Q, K, V: [N, d_model] (or [B, N, d_model]) fp32 on the GPU.
    out (additive): a contiguous fp32 tensor of Q's shape on Q's device to write the result into
    (the batch-shard path writes each rank's rows straight into the gathered result)."""
    if not (Q.is_cuda and K.is_cuda and V.is_cuda):
        raise RuntimeError("Inputs must be CUDA tensors")
    for name, t in (("Q", Q), ("K", K), ("V", V)):
        if t.dtype != torch.float32:
            raise RuntimeError(f"{name} must be float32")
    Qc, Kc, Vc = Q.contiguous(), K.contiguous(), V.contiguous()
    d_model, num_heads = int(d_model), int(num_heads)
    B, N = _shape(Qc, d_model)
    if Kc.shape != Qc.shape or Vc.shape != Qc.shape:
        raise RuntimeError("Q, K and V must have the same shape")
    if kernel not in _lib.VARIANTS:
        warnings.warn(f"Kernel selection supports {sorted(_lib.VARIANTS)}; '{kernel}' routing to default "
                      f"'{_lib.DEFAULT_KERNEL}'")
        kernel = _lib.DEFAULT_KERNEL
    if out is None:
        out = torch.empty_like(Qc)
    elif (out.shape != Qc.shape or out.dtype != torch.float32 or out.device != Qc.device
          or not out.is_contiguous()):
        raise RuntimeError("out must be a contiguous float32 tensor of Q's shape on Q's device")
    lib = _lib.load()
    with torch.cuda.device(Qc.device):
        stream = torch.cuda.current_stream(Qc.device).cuda_stream
        st = lib.qmha_solve_ex(Qc.data_ptr(), Kc.data_ptr(), Vc.data_ptr(), out.data_ptr(), B, N, d_model,
                               num_heads, _lib.variant_id(kernel), stream)
    _lib.check(st, f"flash_solve({kernel})")
    return out


def quantize_int8(X: torch.Tensor, d_model: int, num_heads: int, layout: int = 0):
    """The INT8 pre-pass as an op: per-32-row-group symmetric int8 of every head.

    Returns (Xi [B, h, N, d] int8 (layout 0) or [B, h, N/32, d, 32] (layout 1, V operand
    order), scales [B, h, N/32] fp32); layout 2: [B, h, N, d] rows with one scale per head slice
    (the fa_tc_int8_pt per-tensor mode), scales [B, h]."""
    if not X.is_cuda or X.dtype != torch.float32:
        raise RuntimeError("X must be a float32 CUDA tensor")
    Xc = X.contiguous()
    B, N = _shape(Xc, d_model)
    d = d_model // num_heads
    if layout in (0, 2):
        Xi = torch.empty((B, num_heads, N, d), dtype=torch.int8, device=X.device)
    else:
        Xi = torch.empty((B, num_heads, N // 32, d, 32), dtype=torch.int8, device=X.device)
    sc = torch.empty((B, num_heads) if layout == 2 else (B, num_heads, N // 32), dtype=torch.float32, device=X.device)
    with torch.cuda.device(Xc.device):
        stream = torch.cuda.current_stream(Xc.device).cuda_stream
        st = _lib.load().qmha_quantize_int8(Xc.data_ptr(), B, N, d_model, num_heads, Xi.data_ptr(), sc.data_ptr(),
                                            layout, stream)
    _lib.check(st, "quantize_int8")
    return Xi, sc


def debug_qk_int32(Q: torch.Tensor, K: torch.Tensor, d_model: int, num_heads: int, head: int) -> torch.Tensor:
    """int32 S = Q_i8 K_i8^T of one head through the INT8 path's MFMA operand path (test hook)."""
    if not (Q.is_cuda and K.is_cuda):
        raise RuntimeError("Inputs must be CUDA tensors")
    Qc, Kc = Q.contiguous(), K.contiguous()
    N = Qc.numel() // d_model
    S = torch.empty((N, N), dtype=torch.int32, device=Q.device)
    torch.cuda.synchronize(Q.device)
    with torch.cuda.device(Qc.device):
        st = _lib.load().qmha_debug_qk_int32(Qc.data_ptr(), Kc.data_ptr(), N, d_model, num_heads, head, S.data_ptr())
    _lib.check(st, "debug_qk_int32")
    return S


def debug_fa_int8_dump(Q: torch.Tensor, K: torch.Tensor, V: torch.Tensor, d_model: int, num_heads: int,
                       per_tensor: bool = False):
    """Run the production int8 kernel with its FL_DUMP stores (test hook): returns (O, S, Qi, sQ)
    with O as flash_solve computes it, S [B, h, N, N] int32 = the kernel's own Q@K^T
    accumulators (bias removed), Qi [B, h, N, d] its in-register int8 Q operand, sQ [B, h, N/32].
    per_tensor: the fa_tc_int8_pt kernel instead (sQ then repeats the head slice's one scale)."""
    if not (Q.is_cuda and K.is_cuda and V.is_cuda):
        raise RuntimeError("Inputs must be CUDA tensors")
    Qc, Kc, Vc = Q.contiguous(), K.contiguous(), V.contiguous()
    B, N = _shape(Qc, d_model)
    d = d_model // num_heads
    O = torch.empty_like(Qc)
    S = torch.empty((B, num_heads, N, N), dtype=torch.int32, device=Q.device)
    Qi = torch.empty((B, num_heads, N, d), dtype=torch.int8, device=Q.device)
    sQ = torch.empty((B, num_heads, N // 32), dtype=torch.float32, device=Q.device)
    torch.cuda.synchronize(Q.device)
    with torch.cuda.device(Qc.device):
        lib = _lib.load()
        fn = lib.qmha_debug_fa_int8_pt_dump if per_tensor else lib.qmha_debug_fa_int8_dump
        st = fn(Qc.data_ptr(), Kc.data_ptr(), Vc.data_ptr(), O.data_ptr(), B, N, d_model, num_heads, S.data_ptr(),
                Qi.data_ptr(), sQ.data_ptr())
    _lib.check(st, "debug_fa_int8_dump")
    return O, S, Qi, sQ
