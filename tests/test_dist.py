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
        # per-rank shards (no rank holds the global batch), all-gather overlapped per chunk
        sh = [t[start:stop].clone() for t in (Q, K, V)]
        outs = {c: solve_sharded(*sh, 128, 2, kernel, batch=B, chunks=c, solve_fn=_oracle_solve(oracle))
                for c in (1, 2, 3)}
        mine = solve_sharded(*sh, 128, 2, kernel, batch=B, gather=False, solve_fn=_oracle_solve(oracle))
        assert torch.equal(mine, local)
        with pytest.raises(ValueError):  # a shard of the wrong size is refused, not mis-gathered
            solve_sharded(Q, K, V, 128, 2, kernel, batch=B, solve_fn=_oracle_solve(oracle))
        # the result is written in place (no staging copy): a caller-provided buffer comes back
        buf = torch.empty(B, 64, 128)
        res = solve_sharded(*sh, 128, 2, kernel, batch=B, chunks=3, solve_fn=_oracle_solve(oracle), out=buf)
        assert res.data_ptr() == buf.data_ptr() and torch.equal(res, outs[3])
        # every rank holds the same gathered result: compare against rank 0's through a broadcast
        ref0 = out.clone()
        dist.broadcast(ref0, 0)
        assert torch.equal(ref0, out)
        if rank == 0:
            torch.save({"out": out, **{f"chunked{c}": o for c, o in outs.items()}}, result_path)
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,B,kernel", [(2, 4, "fa_tc_int8_b"), (2, 3, "fa"), (4, 7, "fa_tc_int8_b"),
                                            (4, 10, "fa_tc_v1a")])
def test_shard_gloo(oracle_mod, tmp_path, world, B, kernel):
    """world 2 and 4, even and uneven shards (B = 7 over 4 ranks: 2, 2, 2, 1; B = 10: 3, 3, 2, 2),
    1 / 2 / 3 chunks: every rank's gathered result equals the unsharded computation exactly."""
    path = str(tmp_path / "out.pt")
    mp.start_processes(_worker, args=(world, _free_port(), B, kernel, path), nprocs=world, join=True,
                       start_method="spawn")
    res = torch.load(path, weights_only=True)
    Q, K, V = _inputs(B, 64, 128)
    ref = _oracle_solve(oracle_mod)(Q, K, V, 128, 2, kernel)
    for key, out in res.items():
        assert out.shape == (B, 64, 128), key
        assert torch.equal(out, ref), key  # sharding is exact: the same per-sequence computation


def _subgroup_worker(rank, world, port, B, result_path):
    """World-4 job; ranks 1 and 3 form a subgroup and run the batch-shard path on it (round-3
    ADVICE: P2POp peers must be ranks inside the group, not global ranks)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sub = dist.new_group([1, 3])  # every rank takes part in creating the group
        if rank in (1, 3):
            from oracle import oracle
            Q, K, V = _inputs(B, 64, 128, seed=11)
            r_sub = dist.get_rank(sub)
            start, stop = batch_shard(B, r_sub, 2)
            sh = [t[start:stop].clone() for t in (Q, K, V)]
            outs = {f"chunks{c}": solve_sharded(*sh, 128, 2, "fa_tc_int8_b", batch=B, chunks=c, group=sub,
                                                 solve_fn=_oracle_solve(oracle)) for c in (1, 2)}
            outs["full"] = solve_sharded(Q, K, V, 128, 2, "fa_tc_int8_b", group=sub, solve_fn=_oracle_solve(oracle))
            own = _oracle_solve(oracle)(*sh, 128, 2, "fa_tc_int8_b")
            outs["gather_outputs"] = gather_outputs(own, B, group=sub)
            torch.save(outs, f"{result_path}.{rank}")
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_shard_gloo_subgroup(oracle_mod, tmp_path):
    """The `group=` argument with a subgroup whose members are not global ranks 0..W-1 (ranks 1 and 3
    of a world-4 job): both members end with the full, exact result (even and uneven shards)."""
    for B in (4, 5):
        path = str(tmp_path / f"sub{B}.pt")
        mp.start_processes(_subgroup_worker, args=(4, _free_port(), B, path), nprocs=4, join=True,
                           start_method="spawn")
        Q, K, V = _inputs(B, 64, 128, seed=11)
        ref = _oracle_solve(oracle_mod)(Q, K, V, 128, 2, "fa_tc_int8_b")
        for r in (1, 3):
            res = torch.load(f"{path}.{r}", weights_only=True)
            for key, out in res.items():
                assert out.shape == (B, 64, 128), (r, key)
                assert torch.equal(out, ref), (B, r, key)


def test_bench_spawns_ranks_dry_run():
    """`python bench.py --gpus 2` with no launcher spawns its own two ranks (torch.distributed.run,
    127.0.0.1); --dry-run runs the plumbing on CPU/gloo.  Rank 0 prints one JSON line with
    n_gpus == 2 and the chunked all-gather timing."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "2",
                        "--warmup", "1"], capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["dry_run"] is True and j["value"] is None
    assert j["config"]["global_batch"] == 2 * j["config"]["B_per_gpu"]
    assert j["allgather"]["step_with_allgather_ms"] > 0
    # a launcher/--gpus mismatch is an error, not a silently mislabelled line
    env2 = dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r2 = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                        capture_output=True, text=True, timeout=120, env=env2, cwd=root)
    assert r2.returncode == 2 and "--gpus 2" in r2.stderr


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
def test_bench_torchrun_world1_gpu(tmp_path):
    """The multi-GPU entry point on the GPU: torch.distributed.run, one rank, RCCL process
    group, the HIP kernel, the all-gather legs (compute-only and chunked compute+gather)."""
    import json
    import subprocess
    import sys
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", f"--master-port={_free_port()}", os.path.join(root, "bench.py"), "--gpus", "1", "--steps", "2",
           "--warmup", "1", "--B", "2", "--N", "512", "--no-siblings", "--no-cpu-baseline", "--no-refconfig"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert j["n_gpus"] == 1 and j["value"] > 0
    assert j["allgather"]["allgather_ms"] > 0 and j["allgather"]["value_with_allgather"] > 0


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


def _gpu_worker(rank, world, port, B, result_path):
    """One rank of a world-2 job on the box's single GPU: the HIP kernel computes this rank's
    shard on cuda:0; the all-gather runs over gloo on host copies (RCCL needs one GPU per rank)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from quantizedmha_amd import torch_ext
        dev = torch.device("cuda:0")

        def solve_fn(Q, K, V, d_model, h, kernel):
            return torch_ext.flash_solve(Q.to(dev), K.to(dev), V.to(dev), d_model, h, kernel).cpu()

        Q, K, V = _inputs(B, 256, 256)
        start, stop = batch_shard(B, rank, world)
        sh = [t[start:stop].clone() for t in (Q, K, V)]
        outs = {f"int8_chunks{c}": solve_sharded(*sh, 256, 4, "fa_tc_int8_b", batch=B, chunks=c, solve_fn=solve_fn)
                for c in (1, 2)}
        outs["fp16"] = solve_sharded(*sh, 256, 4, "fa_tc_v1a", batch=B, solve_fn=solve_fn)
        if rank == 0:
            torch.save(outs, result_path)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("B", [4, 5])
def test_shard_hip_world2(tmp_path, B):
    """The batch-shard path with world > 1 driving the HIP kernels: two ranks (gloo), each
    computing its own shard with flash_solve on the GPU, chunked all-gather; the gathered
    output equals one unsharded launch bit for bit (even and uneven shards)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    path = str(tmp_path / "out.pt")
    env_keep = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    try:
        mp.start_processes(_gpu_worker, args=(2, _free_port(), B, path), nprocs=2, join=True, start_method="spawn")
    finally:
        if env_keep is None:
            os.environ.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)
    res = torch.load(path, weights_only=True)
    from quantizedmha_amd import torch_ext
    dev = torch.device("cuda:0")
    Q, K, V = (t.to(dev) for t in _inputs(B, 256, 256))
    ref8 = torch_ext.flash_solve(Q, K, V, 256, 4, "fa_tc_int8_b").cpu()
    ref16 = torch_ext.flash_solve(Q, K, V, 256, 4, "fa_tc_v1a").cpu()
    for key, out in res.items():
        assert out.shape == (B, 256, 256), key
        assert torch.equal(out, ref16 if key == "fp16" else ref8), key
