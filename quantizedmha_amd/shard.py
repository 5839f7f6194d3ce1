"""Batch-shard execution across GPUs (BASELINE config 5).

Every (sequence, head) pair of the attention forward is independent, so the multi-GPU path is
a pure partition of the batch: rank r of W owns sequences [start_r, stop_r) and runs the
single-GPU kernel on them with no data-path collective.  The north star's RCCL all-gather of
the per-shard outputs over xGMI is a separate, optional step; outputs are batch-outermost
[B, N, d_model], so every rank's shard is one contiguous slab of the result.  With
`chunks > 1` the shard is computed in batch chunks and the all-gather of chunk c runs on the
collective's own stream while chunk c+1 is being computed (the gather is ~1/3 of the compute
at C5 over one xGMI link per peer, so only the last chunk's gather is exposed).

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm; "gloo" for CPU tests).
Each rank only ever holds its own shard of Q/K/V (`batch=` form of `solve_sharded`), so the
per-GPU memory is that of the single-GPU C4 problem whatever the global batch.
The reference has no multi-GPU code; this module is the build's addition.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple

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


def _world(group) -> Tuple[int, int]:
    if not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def _padded(O: torch.Tensor, width: int) -> torch.Tensor:
    if O.shape[0] == width:
        return O.contiguous()
    pad = O.new_zeros((width - O.shape[0],) + tuple(O.shape[1:]))
    return torch.cat([O, pad], 0)


def _trim(buf: torch.Tensor, batch: int, world: int, width: int) -> torch.Tensor:
    sizes = [batch_shard(batch, r, world) for r in range(world)]
    if all(stop - start == width for start, stop in sizes):
        return buf
    return torch.cat([buf[r * width:r * width + (stop - start)] for r, (start, stop) in enumerate(sizes)], 0)


def gather_outputs(O_local: torch.Tensor, batch: int, group=None) -> torch.Tensor:
    """All-gather per-rank outputs [b_r, N, d_model] into the full [batch, N, d_model] on every
    rank.  Uneven shards are padded to the largest shard for the collective and trimmed."""
    world, _ = _world(group)
    if world == 1:
        return O_local
    width = max(stop - start for start, stop in (batch_shard(batch, r, world) for r in range(world)))
    O_send = _padded(O_local, width)
    buf = O_send.new_empty((world * width,) + tuple(O_send.shape[1:]))
    dist.all_gather_into_tensor(buf, O_send, group=group)
    return _trim(buf, batch, world, width)


def solve_shard_gather(Q: torch.Tensor, K: torch.Tensor, V: torch.Tensor, d_model: int, num_heads: int,
                       batch: int, kernel: str = "fa_tc_int8_b", group=None, chunks: int = 1,
                       solve_fn: Optional[Callable] = None) -> torch.Tensor:
    """This rank's shard [b_r, N, d_model] in; the full [batch, N, d_model] out on every rank.

    The shard is computed in `chunks` batch chunks; chunk c's all-gather is issued
    asynchronously right after its compute is enqueued, so it overlaps chunk c+1's kernels
    (RCCL orders it after chunk c on the compute stream by itself).  Chunk boundaries are the
    same on every rank (chunks of the padded shard width), so each collective moves equal
    sizes; a rank with a short shard contributes zero padding that is trimmed at the end."""
    world, rank = _world(group)
    lo, hi = batch_shard(batch, rank, world)
    if Q.shape[0] != hi - lo:
        raise ValueError(f"rank {rank} of {world}: expected its shard of {hi - lo} sequences, got {Q.shape[0]}")
    if solve_fn is None:
        from .torch_ext import flash_solve as solve_fn  # HIP path; raises if the library is absent
    width = max(stop - start for start, stop in (batch_shard(batch, r, world) for r in range(world)))
    if world == 1:
        return solve_fn(Q, K, V, d_model, num_heads, kernel)
    C = max(1, min(int(chunks), width))
    buf = Q.new_empty((world * width,) + tuple(Q.shape[1:]))
    works: List = []
    keep: List[torch.Tensor] = []
    for c in range(C):
        c0, c1 = batch_shard(width, c, C)
        n = max(0, min(c1, Q.shape[0]) - c0)
        if n > 0:
            O_c = solve_fn(Q[c0:c0 + n], K[c0:c0 + n], V[c0:c0 + n], d_model, num_heads, kernel)
        else:
            O_c = Q.new_empty((0,) + tuple(Q.shape[1:]))
        O_c = _padded(O_c, c1 - c0)
        views = [buf[r * width + c0:r * width + c1] for r in range(world)]
        works.append(dist.all_gather(views, O_c, group=group, async_op=True))
        keep.append(O_c)
    for w in works:
        w.wait()
    return _trim(buf, batch, world, width)


def solve_sharded(Q: torch.Tensor, K: torch.Tensor, V: torch.Tensor, d_model: int, num_heads: int,
                  kernel: str = "fa_tc_int8_b", gather: bool = True, group=None,
                  solve_fn: Optional[Callable] = None, batch: Optional[int] = None,
                  chunks: int = 1) -> torch.Tensor:
    """Batch-sharded attention forward.

    batch=None: Q, K, V are the FULL batch [B, N, d_model] (or views of it) and rank r slices
    its shard.  batch=B: Q, K, V are already this rank's shard (`batch_shard(B, r, W)`), which
    is how a real C5 job holds its inputs (no rank ever materialises the global batch).
    Rank r computes its shard with `solve_fn` (default: torch_ext.flash_solve, the HIP
    kernels) and, if `gather`, returns the full [B, N, d_model] output on every rank
    (all-gather overlapped with compute when chunks > 1), else its own shard.
    """
    if Q.dim() != 3:
        raise ValueError("solve_sharded expects [B, N, d_model] inputs")
    if solve_fn is None:
        from .torch_ext import flash_solve as solve_fn  # HIP path; raises if the library is absent
    world, rank = _world(group)
    if batch is None:
        batch = Q.shape[0]
        start, stop = batch_shard(batch, rank, world)
        Q, K, V = Q[start:stop], K[start:stop], V[start:stop]
    if not gather or world == 1:
        lo, hi = batch_shard(batch, rank, world)
        if Q.shape[0] != hi - lo:
            raise ValueError(f"rank {rank} of {world}: expected its shard of {hi - lo} sequences, got {Q.shape[0]}")
        return solve_fn(Q, K, V, d_model, num_heads, kernel)
    return solve_shard_gather(Q, K, V, d_model, num_heads, batch, kernel, group, chunks, solve_fn)
