"""Multi-process (gloo, world size 2, CPU) coverage of the env-sharded path:
shard bounds, per-rank seeds, max-over-ranks timing and the per-episode stats
all-gather -- and that stepping the C4 scenario shard by shard (oracle on the
CPU) reproduces the unsharded batch, i.e. envs really are independent."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from powergridworld_amd.distributed import (gather_episode_stats, max_over_ranks, rank_seed,
                                            shard_bounds)

K, STEPS = 12, 6


def test_shard_bounds_cover_and_balance():
    for total in (0, 1, 7, 65536, 524288 + 3):
        for world in (1, 2, 3, 8):
            shards = [shard_bounds(total, r, world) for r in range(world)]
            assert shards[0].start == 0 and shards[-1].stop == total
            for a, b in zip(shards, shards[1:]):
                assert a.stop == b.start
            assert max(s.count for s in shards) - min(s.count for s in shards) <= 1
    assert shard_bounds(524288, 7, 8).count == 65536
    seeds = {rank_seed(0, r, a) for r in range(8) for a in range(5)}
    assert len(seeds) == 40
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


def _c4_oracle(init_soc, acts):
    from oracle.ma_oracle import CoordinatedOracle
    orc = CoordinatedOracle(init_soc.shape[1])
    obs0 = orc.reset(init_soc)
    rew, vv, obs = [], [], [obs0]
    for a in acts:
        o, r, v = orc.step(a)
        obs.append(o)
        rew.append(r)
        vv.append(v)
    return np.stack(obs), np.stack(rew), np.stack(vv)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(0)
        init_soc = rng.uniform(3, 50, (5, K))                 # the global batch, same on every rank
        acts = rng.uniform(-1, 1, (STEPS, 5, K, 8))
        sh = shard_bounds(K, rank, world)
        obs, rew, vv = _c4_oracle(init_soc[:, sh.start:sh.stop], acts[:, :, sh.start:sh.stop])
        # per-env episode statistics, gathered once per episode in global env order
        ep = torch.from_numpy(np.concatenate([rew.sum(0).T, vv.sum(0)[:, None]], 1))
        allep = gather_episode_stats(ep)
        t = max_over_ranks(0.5 + rank)
        if rank == 0:
            q.put((allep.numpy(), t))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_c4_equals_unsharded_gloo_ws2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, t = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == 1.5                                           # max over ranks
    rng = np.random.default_rng(0)
    init_soc = rng.uniform(3, 50, (5, K))
    acts = rng.uniform(-1, 1, (STEPS, 5, K, 8))
    _, rew, vv = _c4_oracle(init_soc, acts)
    want = np.concatenate([rew.sum(0).T, vv.sum(0)[:, None]], 1)
    assert got.shape == want.shape == (K, 6)
    # per-env results do not depend on the batch they run in (BLAS blocking may
    # differ by batch size, so not necessarily bitwise)
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12)

