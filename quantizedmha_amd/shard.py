"""Batch-shard execution across GPUs (BASELINE config 5).

Every (sequence, head) pair of the attention forward is independent, so the multi-GPU path is
a pure partition of the batch: rank r of W owns sequences [start_r, stop_r) and runs the
single-GPU kernel on them with no data-path collective.  The north star's RCCL all-gather of
the per-shard outputs over xGMI is a separate, optional step (`gather_outputs`); outputs are
batch-outermost [B, N, d_model], so every rank's shard is one contiguous slab of the result.

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm; "gloo" for CPU tests).
The reference has no multi-GPU code; this module is the build's addition.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


def batch_shard(batch: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [start, stop) of the batch owned by `rank`; the first batch % world ranks
    get one extra sequence, so shard sizes differ by at most one."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"invalid rank {rank} of world {world}")
    if batch < 0:
        raise ValueError(f"invalid batch {batch}")
    base, extra = divmod(batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_outputs(O_local: torch.Tensor, batch: int, group=None) -> torch.Tensor:
    """All-gather per-rank outputs [b_r, N, d_model] into the full [batch, N, d_model] on every
    rank.  Uneven shards are padded to the largest shard for the collective and trimmed."""
    world = dist.get_world_size(group)
    if world == 1:
        return O_local
    sizes = [batch_shard(batch, r, world) for r in range(world)]
    width = max(stop - start for start, stop in sizes)
    if O_local.shape[0] != width:
        pad = O_local.new_zeros((width - O_local.shape[0],) + tuple(O_local.shape[1:]))
        O_send = torch.cat([O_local, pad], 0)
    else:
        O_send = O_local.contiguous()
    buf = O_send.new_empty((world * width,) + tuple(O_send.shape[1:]))
    dist.all_gather_into_tensor(buf, O_send, group=group)
    if all(stop - start == width for start, stop in sizes):
        return buf
    return torch.cat([buf[r * width:r * width + (stop - start)] for r, (start, stop) in enumerate(sizes)], 0)


def solve_sharded(Q: torch.Tensor, K: torch.Tensor, V: torch.Tensor, d_model: int, num_heads: int,
                  kernel: str = "fa_tc_int8_b", gather: bool = True, group=None,
                  solve_fn: Optional[Callable] = None) -> torch.Tensor:
    """Batch-sharded attention forward.

    Q, K, V: the FULL batch [B, N, d_model] (each rank may hold it, or a view of it); rank r
    computes its shard with `solve_fn` (default: torch_ext.flash_solve, the HIP kernels) and,
    if `gather`, returns the full [B, N, d_model] output on every rank, else its own shard.
    """
    if Q.dim() != 3:
        raise ValueError("solve_sharded expects [B, N, d_model] inputs")
    if solve_fn is None:
        from .torch_ext import flash_solve as solve_fn  # HIP path; raises if the library is absent
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    start, stop = batch_shard(Q.shape[0], rank, world)
    O_local = solve_fn(Q[start:stop], K[start:stop], V[start:stop], d_model, num_heads, kernel)
    if not gather or world == 1:
        return O_local
    return gather_outputs(O_local, Q.shape[0], group)
