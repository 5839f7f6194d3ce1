"""Batch-shard execution across GPUs (BASELINE config 5).

Every (sequence, head) pair of the attention forward is independent, so the multi-GPU path is
a pure partition of the batch: rank r of W owns sequences [start_r, stop_r) and runs the
single-GPU kernel on them with no data-path collective.  The north star's RCCL all-gather of
the per-shard outputs over xGMI is a separate, optional step; outputs are batch-outermost
[B, N, d_model], so every rank's shard is one contiguous slab of the result: each rank's
kernels write their rows straight into the result tensor and the gather is a point-to-point
exchange into the peers' slabs (no staging buffer, no reorder copy).  With `chunks > 1` the
shard is computed in batch chunks and the exchange of chunk c runs on the collective's own
stream while chunk c+1 is being computed.

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
                       solve_fn: Optional[Callable] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """This rank's shard [b_r, N, d_model] in; the full [batch, N, d_model] out on every rank.

    Copy-free: the result tensor `out` is allocated once (or passed in) and every rank's kernels
    write their rows straight into their own slab of it (flash_solve(out=...)).  The exchange is
    point-to-point: for each batch chunk c, every rank sends its chunk-c rows to each peer and
    receives each peer's chunk-c rows straight into that peer's slab (one isend / irecv pair per
    peer, batched in one RCCL group).  On the MI355X node's xGMI full mesh every peer's data
    travels on its own link, and nothing is staged, padded or reordered: uneven shards just send
    fewer rows.  Chunk c's exchange is issued right after chunk c's kernels are enqueued, so it
    runs on the collective stream while chunk c+1 computes; chunk boundaries (chunks of the
    largest shard's width) are the same on every rank, so sends and receives pair up.  Peers are
    addressed by their rank INSIDE `group` (P2POp's group_peer; its positional `peer` is a global
    rank), so a subgroup whose members are not global ranks 0..W-1 exchanges correctly.

    solve_fn (CPU tests: the oracle) returns a new tensor that is copied into the slab; the
    default HIP path writes in place."""
    world, rank = _world(group)
    lo, hi = batch_shard(batch, rank, world)
    if Q.shape[0] != hi - lo:
        raise ValueError(f"rank {rank} of {world}: expected its shard of {hi - lo} sequences, got {Q.shape[0]}")
    if out is None:
        out = Q.new_empty((batch,) + tuple(Q.shape[1:]))
    elif out.shape != (batch,) + tuple(Q.shape[1:]) or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous {(batch,) + tuple(Q.shape[1:])} tensor")

    def compute(q, k, v, dst):
        if solve_fn is None:
            from .torch_ext import flash_solve  # HIP path; raises if the library is absent
            flash_solve(q, k, v, d_model, num_heads, kernel, out=dst)
        else:
            dst.copy_(solve_fn(q, k, v, d_model, num_heads, kernel))

    if world == 1:
        compute(Q, K, V, out)
        return out
    sizes = [batch_shard(batch, r, world) for r in range(world)]
    width = max(stop - start for start, stop in sizes)
    C = max(1, min(int(chunks), width))
    works: List = []
    for c in range(C):
        c0, c1 = batch_shard(width, c, C)
        n = max(0, min(c1, hi - lo) - c0)
        mine = out[lo + c0:lo + c0 + n]
        if n > 0:
            compute(Q[c0:c0 + n], K[c0:c0 + n], V[c0:c0 + n], mine)
        ops = []
        for p, (ps, pe) in enumerate(sizes):
            if p == rank:
                continue
            if n > 0:
                ops.append(dist.P2POp(dist.isend, mine, group=group, group_peer=p))
            n_p = max(0, min(c1, pe - ps) - c0)
            if n_p > 0:
                ops.append(dist.P2POp(dist.irecv, out[ps + c0:ps + c0 + n_p], group=group, group_peer=p))
        if ops:
            works.extend(dist.batch_isend_irecv(ops))
    for w in works:
        w.wait()
    return out


def solve_sharded(Q: torch.Tensor, K: torch.Tensor, V: torch.Tensor, d_model: int, num_heads: int,
                  kernel: str = "fa_tc_int8_b", gather: bool = True, group=None,
                  solve_fn: Optional[Callable] = None, batch: Optional[int] = None,
                  chunks: int = 1, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Batch-sharded attention forward.

    batch=None: Q, K, V are the FULL batch [B, N, d_model] (or views of it) and rank r slices
    its shard.  batch=B: Q, K, V are already this rank's shard (`batch_shard(B, r, W)`), which
    is how a real C5 job holds its inputs (no rank ever materialises the global batch).
    Rank r computes its shard with `solve_fn` (default: torch_ext.flash_solve, the HIP
    kernels) and, if `gather`, returns the full [B, N, d_model] output on every rank
    (point-to-point exchange overlapped with compute when chunks > 1; written into `out` when
    given), else its own shard.
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
    return solve_shard_gather(Q, K, V, d_model, num_heads, batch, kernel, group, chunks, solve_fn, out)
