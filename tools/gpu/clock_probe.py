"""Probe: k_mc_step's cost per clock mode on C3 (16 384 envs, full episodes):
eager without the device clock (CLK 0), eager with it (CLK 1), and the
captured step reading the device table (CLK 2).  Run under rocprofv3
--kernel-trace; prints wall us/step per mode."""
import json
import os
import sys
import time

import torch

ROOT = os.environ.get("GRAFT_REPO_ROOT", ".")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench_configs import c3_env  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
n, pool = 16384, 16
env, acts = c3_env(dev, n, pool)
init = torch.full((n,), 30.0, dtype=torch.float64, device=dev)
graphs = None


def episode(mode):
    global graphs
    env.reset(init_storage=init)
    if mode == 2 and graphs is None:
        graphs = [env.capture_step(a) for a in acts]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(286):
        if mode == 2:
            graphs[k % pool]()
        else:
            env.step(acts[k % pool])
            if mode == 0 and k == 0:
                env._mc_args.clock = None          # (CLK 0 from the second step)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / 286 * 1e6


for mode in (0, 1, 2, 0, 1, 2):
    us = episode(mode)
    env._mc_args = None                          # rebuilt (with the clock) at the next step
    print(json.dumps({"clk": mode, "us_per_step": us}), flush=True)
