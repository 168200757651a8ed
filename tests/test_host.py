"""Host-side logic (CPU): synthetic workloads, sharding, and the multi-rank
reduction path of bench.py over gloo (world_size 2)."""
import os
import socket

import numpy as np
import pytest

from trajopt_amd import problems, robots, sharding


def test_splitmix64_known_values():
    """splitmix64 reference sequence for seed 0 (Vigna's published outputs)."""
    r = problems.SplitMix64(0)
    assert [r.next() for _ in range(3)] == [0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4, 0x06C45D188009454F]


def test_workload_deterministic_and_seeded_per_problem():
    a = problems.make_workload("B", 4)
    b = problems.make_workload("B", 4)
    np.testing.assert_array_equal(a.init, b.init)
    np.testing.assert_array_equal(a.targets, b.targets)
    # problem k of a batch is independent of the batch it is generated in
    c = problems.make_workload("B", 2, first_problem=2)
    np.testing.assert_array_equal(a.init[2:], c.init)
    np.testing.assert_array_equal(a.targets[2:], c.targets)


def test_workload_shapes_and_limits():
    for cfg, N, ncart in (("A", 10, 1), ("B", 30, 29)):
        wl = problems.make_workload(cfg, 3)
        assert wl.init.shape == (3, N, 7)
        assert wl.targets.shape == (3, ncart, 12)
        lo, hi, _ = robots.chain_limits(wl.desc.chain)
        assert np.all(wl.q_ref >= lo - 1e-12) and np.all(wl.q_ref <= hi + 1e-12)
        # targets are tool poses of q_ref (rotation part orthonormal)
        R = wl.targets[..., [0, 1, 2, 4, 5, 6, 8, 9, 10]].reshape(3, ncart, 3, 3)
        np.testing.assert_allclose(R @ np.swapaxes(R, -1, -2), np.broadcast_to(np.eye(3), R.shape), atol=1e-12)
        # fixed start step is the interpolation start
        np.testing.assert_allclose(wl.init[:, 0], wl.q_ref[:, 0])


def test_shard_ranges_partition_the_seed_space():
    B = 5
    seen = []
    for r in range(4):
        wl = sharding.rank_workload("A", B, r)
        full = problems.make_workload("A", B, first_problem=sharding.shard_first(r, B))
        np.testing.assert_array_equal(wl.init, full.init)
        seen.extend(range(sharding.shard_first(r, B), sharding.shard_first(r, B) + B))
    assert seen == list(range(4 * B))
    with pytest.raises(ValueError):
        sharding.shard_first(-1, 4)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q):
    import sys
    from pathlib import Path

    repo = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(repo), str(repo / "trajopt-1_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    from oracle import oracle  # CPU checker stands in for the device solve here
    from trajopt_amd import sharding as sh

    dist.init_process_group("gloo", rank=rank, world_size=world)
    wl = sh.rank_workload("A", 3, rank)
    x, res = oracle.solve(wl, n_threads=1)
    iters = sum(r.n_sqp_iters for r in res)
    elapsed = 0.5 + rank  # synthetic per-rank times: the reduction must take the max
    tmax, itot = sh.reduce_step_stats(elapsed, iters, world)
    q.put((rank, x, [r.status for r in res], iters, tmax, itot))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_sharding_matches_single_process(oracle_mod):
    """bench.py's N>1 path: each rank solves its own seed range; the union of
    the shards equals the single-process batch; max-time / sum-iterations
    reductions are correct."""
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort(key=lambda t: t[0])
    full = problems.make_workload("A", 3 * world)
    xf, rf = oracle_mod.solve(full, n_threads=2)
    x = np.concatenate([o[1] for o in out])
    np.testing.assert_allclose(x, xf, rtol=0, atol=0)
    assert [s for o in out for s in o[2]] == [r.status for r in rf]
    total = sum(r.n_sqp_iters for r in rf)
    for o in out:
        assert o[4] == 0.5 + (world - 1)
        assert o[5] == total
