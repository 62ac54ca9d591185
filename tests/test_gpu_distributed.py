"""The env-sharded device path across ranks: two gloo ranks,
both on cuda:0, each step their shard_bounds slice of C4 (OpenDSS rule, fused
pgw_coord_step) through the public API; every per-env output equals the
unsharded batch's bit for bit, and the per-episode statistics come back in
global env order through gather_episode_stats on device tensors, the step time
through max_over_ranks.  The ranks are forked from the forkserver conftest.py
starts before this process touches the GPU (no exec of, and no fork from, a
GPU-initialised process).  Needs an MI355X.  Multi-GPU runs (RCCL over xGMI)
are the driver's: unmeasured here."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
K, STEPS, WORLD = 320, 24, 2


def _run_c4(start, stop, seed_env):
    """Steps envs [start, stop) of the global batch; returns per-step rewards
    [T, 5, n], violations [T, n], V675.3 [T, n], iterations [T, n] (device) and
    the per-env episode statistics [n, 6] (device)."""
    from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config
    dev = torch.device("cuda:0")
    g = np.load(os.path.join(HERE, "golden", "c4_two_episodes.npz"))
    Kg = g["actions"].shape[3]
    idx = np.arange(start, stop) % Kg
    env = CoordinatedMultiBuildingControlEnv(**make_c4_config(pf_convergence="opendss"), num_envs=stop - start,
                                             device=dev, fused=True)
    T = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)
    env.reset()
    for a, agent in enumerate(env.agents):
        agent.env_dict["storage"].reset(init_storage=T(g["init_storage"][0, a][idx]))
    env.load_component_state()
    rew, vv, v, it = [], [], [], []
    for t in range(STEPS):
        _, r, _, meta = env.step(T(g["actions"][0, t][:, idx]))
        rew.append(torch.stack([r[a.name] for a in env.agents]).clone())
        vv.append(meta["voltage_violation"].clone())
        v.append(env.pf_solver.get_bus_voltage_by_name("675c").clone())
        it.append(env.pf_solver.iterations.clone())
    rew, vv = torch.stack(rew), torch.stack(vv)
    stats = torch.cat([rew.sum(0).T, vv.sum(0)[:, None]], 1)
    return rew, vv, torch.stack(v), torch.stack(it), stats


def _rank(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    from powergridworld_amd import distributed as pgd
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        torch.cuda.set_device(0)
        sh = pgd.shard_bounds(K, rank, WORLD)
        rew, vv, v, it, stats = _run_c4(sh.start, sh.stop, rank)
        torch.cuda.synchronize()
        allstats = pgd.gather_episode_stats(stats)          # device tensor in, device tensor out
        t = pgd.max_over_ranks(1.0 + rank, torch.device("cuda:0"))
        assert allstats.device.type == "cuda" and allstats.shape == (K, 6)
        q.put((rank, sh.start, sh.stop, rew.cpu().numpy(), vv.cpu().numpy(), v.cpu().numpy(),
               it.cpu().numpy(), allstats.cpu().numpy() if rank == 0 else None, t))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_gloo_ranks_on_one_gpu_equal_unsharded_batch():
    if mp.get_all_start_methods().count("forkserver") == 0:
        pytest.skip("no forkserver start method")
    import multiprocessing.forkserver as fs
    if fs._forkserver._forkserver_pid is None:
        pytest.skip("forkserver not started before GPU use (run with -m gpu)")
    ctx = mp.get_context("forkserver")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(WORLD):
        r = q.get(timeout=240)
        got[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rew, vv, v, it, stats = [x.cpu().numpy() for x in _run_c4(0, K, 0)]
    for r in range(WORLD):
        _, a, b, r_rew, r_vv, r_v, r_it, _, t = got[r]
        np.testing.assert_array_equal(r_rew, rew[:, :, a:b])
        np.testing.assert_array_equal(r_vv, vv[:, a:b])
        np.testing.assert_array_equal(r_v, v[:, a:b])
        np.testing.assert_array_equal(r_it, it[:, a:b])
        assert t == float(WORLD)                       # max over ranks of 1.0 + rank
    np.testing.assert_array_equal(got[0][7], stats)     # gathered in global env order
    assert got[0][2] == got[1][1] and got[1][2] == K
