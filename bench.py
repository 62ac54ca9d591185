"""Benchmark: agent-env-steps/sec of the 5-agent coordinated-building scenario
with the IEEE-13 power flow (BASELINE.json config C4), batch 65,536 per GPU.

One "step" = one MultiAgentEnv.step of the whole batch through the public API
(fused path: ONE pgw_coord_step launch: 5 x [building, PV, storage] agents +
power flow + coordinated reward), actions already resident in HBM.  Episodes
(286 steps) end with done["__all__"]; the following env.reset() is inside the
timed region.

Launch:  python bench.py [--gpus N --steps K --warmup W]
         (N>1 via torch.distributed.run: one rank per GPU, weak scaling,
          no collective on the step path; barrier + max-over-ranks timing.)
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

N_AGENTS = 5
ACT_DIM = 8
BATCH_PER_GPU = 65536
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Algorithmic HBM bytes per env-step of pgw_coord_step (fp64, env-minor SoA), per agent:
#   reads  actions 8x8 + x_k 5x8 + soc 8                       = 112
#   writes x_k 5x8 + soc 8 + obs 17x8 + reward 8 + power 8     = 200
# plus per env the bus voltage and the voltage violation (2 x 8).   (1,568)
BYTES_PER_ENV_STEP = N_AGENTS * (112 + 200) + 16


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=572)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--batch", type=int, default=BATCH_PER_GPU)
    ap.add_argument("--action-pool", type=int, default=64,
                    help="distinct pre-generated action batches cycled through (HBM resident)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-envs", type=int, default=2048)
    ap.add_argument("--cpu-sample-steps", type=int, default=30)
    return ap.parse_args()


def cpu_baseline(envs, steps):
    """The oracle (NumPy port of the reference step path) on the host, 1 thread."""
    from threadpoolctl import threadpool_limits
    from oracle.ma_oracle import CoordinatedOracle
    rng = np.random.default_rng(0)
    with threadpool_limits(limits=1):
        orc = CoordinatedOracle(envs)
        orc.reset(rng.uniform(3, 50, (N_AGENTS, envs)))
        acts = [rng.uniform(-1, 1, (N_AGENTS, envs, ACT_DIM)) for _ in range(steps)]
        t0 = time.perf_counter()
        for a in acts:
            orc.step(a)
        dt = time.perf_counter() - t0
    return {"value": N_AGENTS * envs * steps / dt, "unit": "agent-env-steps/s", "cores": 1,
            "kind": "port",
            "sample": "oracle/ma_oracle.CoordinatedOracle (batched NumPy fp64 port of the "
                      "reference step path + PF), %d envs x %d steps, 1 thread, %.1f s"
                      % (envs, steps, dt)}


def load_traffic():
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(p):
        with open(p) as f:
            d = json.load(f)
        return d.get("bytes_per_launch")
    return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from powergridworld_amd.scenarios.coordinated import (CoordinatedMultiBuildingControlEnv,
                                                          make_c4_config)
    n = args.batch
    env = CoordinatedMultiBuildingControlEnv(**make_c4_config(), num_envs=n, device=dev, fused=True)
    for i, agent in enumerate(env.agents):         # per-rank seed offset
        agent.env_dict["storage"].seed(1000 * rank + i)
    gen = torch.Generator(dev).manual_seed(rank)
    P = args.action_pool
    pool = torch.empty((P, N_AGENTS, ACT_DIM, n), dtype=torch.float64, device=dev)
    pool.uniform_(-1.0, 1.0, generator=gen)
    packed = pool.transpose(2, 3)                  # [P, agents, N, act_dim] view, env-minor

    env.reset()
    step_count = 0

    def run(k, events=None):
        nonlocal step_count
        for i in range(k):
            if events is not None:
                events[i][0].record()
            _, _, dones, _ = env.step(packed[step_count % P])
            if events is not None:
                events[i][1].record()
            step_count += 1
            if dones["__all__"]:
                env.reset()

    run(args.warmup)
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps, ev)
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    total_envs = n * world
    value = N_AGENTS * total_envs * args.steps / elapsed
    if rank == 0:
        achieved = BYTES_PER_ENV_STEP * n / (kernel_ms * 1e-3) / 1e9
        traffic = load_traffic()
        out = {
            "metric": "agent-env-steps/sec at batch 65536, 5-agent scenario, 1/2/4/8 MI355X",
            "value": value,
            "unit": "agent-env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded uniform actions pre-generated on device, synthetic "
                    "exogenous building data, IEEE-13 feeder + 8760-h loadshape)",
            "config": {"workload": "C4: 5-agent coordinated buildings (building+PV+storage) "
                                   "+ IEEE-13 power flow + voltage-violation reward",
                       "batch_per_gpu": n, "global_batch": total_envs, "episode_steps": 286,
                       "parallelism": "env-sharded x%d (no collective on the step path)" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "kernel": "pgw_coord_step (k_coord_step<14>)",
                         "kernel_ms": kernel_ms,
                         "bytes_per_launch": BYTES_PER_ENV_STEP * n},
        }
        it = env.pf_solver.iterations
        if it is not None:
            itf = it.double()
            out["pf_iterations"] = {"mean": float(itf.mean()), "max": int(it.max())}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_sample_envs, args.cpu_sample_steps)
        print(json.dumps(out))
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
