"""Probe: host cost of a step launched eagerly vs replayed from a captured
hipGraph (torch.cuda.CUDAGraph over the env's own ctypes launch), for C2
(EnergyStorageEnv, 4096 envs) and C3 (MultiComponentEnv, 16 384 envs).  The
C3 capture freezes the step's per-step arguments (timing only: the replayed
values are those of the captured step); graphs of 1 and of 8 steps."""
import json
import os
import sys
import time

import torch

ROOT = os.environ.get("GRAFT_REPO_ROOT", ".")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench_configs import c3_env  # noqa: E402
from powergridworld_amd.agents import EnergyStorageEnv  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
K = 2000


def timeit(fn, k=K):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    h = time.perf_counter() - t0
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e6, h / k * 1e6


def probe(label, env, step_once, reset):
    out = {}
    reset()
    out["eager_us"], out["eager_host_us"] = timeit(step_once, 200)
    reset()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step_once()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    for steps in (1, 8):
        reset()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(steps):
                step_once()
        torch.cuda.synchronize()
        us, host = timeit(g.replay, K // steps)
        out["graph%d_us_per_step" % steps] = us / steps
        out["graph%d_host_us_per_step" % steps] = host / steps
    print(json.dumps(dict(config=label, **out)), flush=True)


n = 4096
env = EnergyStorageEnv(num_envs=n, device=dev)
act = torch.empty((n, 1), dtype=torch.float64, device=dev).uniform_(-1, 1)
init = torch.full((n,), 30.0, dtype=torch.float64, device=dev)


def c2_step():
    env.step(act)
    if env.simulation_step > 250:
        env.simulation_step = 0


probe("C2", env, c2_step, lambda: env.reset(init_storage=init))

env3, acts = c3_env(dev, 16384, 1)


def c3_step():
    env3.step(acts[0])
    if env3.time_index > 250 if hasattr(env3, "time_index") else False:
        pass


def c3_reset():
    env3.reset(init_storage=init.new_full((16384,), 30.0))


probe("C3", env3, c3_step, c3_reset)
