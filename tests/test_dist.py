"""Multi-process batch-shard path (quantizedmha_amd/shard.py) on CPU with the gloo backend.

The shard compute here is the CPU oracle (the checker), standing in for the HIP kernel so the
partition + all-gather plumbing runs without a GPU; on the GPU box the same code runs with
flash_solve over RCCL (bench.py --gpus N, and test_shard_gpu_world1 below).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from quantizedmha_amd.shard import batch_shard, gather_outputs, solve_sharded


def test_batch_shard_partitions():
    for batch in (0, 1, 3, 16, 17, 128):
        for world in (1, 2, 3, 8):
            ranges = [batch_shard(batch, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == batch
            for (a0, b0), (a1, b1) in zip(ranges, ranges[1:]):
                assert b0 == a1  # contiguous, disjoint
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1
    assert batch_shard(128, 3, 8) == (48, 64)  # BASELINE config 5: 16 sequences per GPU
    with pytest.raises(ValueError):
        batch_shard(4, 2, 2)


def _oracle_solve(oracle_mod):
    def solve(Q, K, V, d_model, h, kernel):
        fn = oracle_mod.ORACLE_BY_VARIANT[kernel]
        outs = [fn(q.numpy(), k.numpy(), v.numpy(), d_model, h, 1) for q, k, v in zip(Q, K, V)]
        return torch.from_numpy(np.stack(outs)) if outs else Q.new_empty((0,) + tuple(Q.shape[1:]))
    return solve


def _inputs(B, N, d_model, seed=7):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(B, N, d_model, generator=g) * 0.5 for _ in range(3)]


def _worker(rank, world, port, B, kernel, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle
        Q, K, V = _inputs(B, 64, 128)
        out = solve_sharded(Q, K, V, 128, 2, kernel, solve_fn=_oracle_solve(oracle))
        local = solve_sharded(Q, K, V, 128, 2, kernel, gather=False, solve_fn=_oracle_solve(oracle))
        start, stop = batch_shard(B, rank, world)
        assert local.shape[0] == stop - start
        if rank == 0:
            torch.save({"out": out}, result_path)
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("B,kernel", [(4, "fa_tc_int8_b"), (3, "fa")])
def test_shard_gloo_world2(oracle_mod, tmp_path, B, kernel):
    path = str(tmp_path / "out.pt")
    mp.start_processes(_worker, args=(2, _free_port(), B, kernel, path), nprocs=2, join=True,
                       start_method="spawn")
    out = torch.load(path, weights_only=True)["out"]
    Q, K, V = _inputs(B, 64, 128)
    ref = _oracle_solve(oracle_mod)(Q, K, V, 128, 2, kernel)
    assert out.shape == (B, 64, 128)
    assert torch.equal(out, ref)  # sharding is exact: the same per-sequence computation


def test_gather_world1_passthrough():
    x = torch.arange(6.0).reshape(1, 2, 3)
    if not dist.is_initialized():
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
        dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        assert gather_outputs(x, 1) is x
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_shard_gpu_world1():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from quantizedmha_amd import torch_ext
    dev = torch.device("cuda:0")
    Q, K, V = (t.to(dev) for t in _inputs(2, 256, 256))
    out = solve_sharded(Q, K, V, 256, 4, "fa_tc_int8_b")
    ref = torch_ext.flash_solve(Q, K, V, 256, 4, "fa_tc_int8_b")
    assert torch.equal(out, ref)
