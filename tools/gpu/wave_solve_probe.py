"""Latency of od_wave_solve (the one-launch C4 step's inline snap solve): the
fused step at 4 096 envs (64 blocks) with every response record forced unfit,
so every wave solves its 64 envs one after another; rocprof/event time per
step / 64 = one solve's latency.  Also the same step with the table serving.
Usage: python tools/gpu/wave_solve_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config  # noqa: E402
from test_gpu_pf_od import _unfit  # noqa: E402


def run(every, n=4096, steps=40):
    env = CoordinatedMultiBuildingControlEnv(**make_c4_config(), num_envs=n, device="cuda", fused=True)
    env.reset()
    if every:
        _unfit(env.pf_solver, every)
    g = torch.Generator("cuda").manual_seed(3)
    acts = [torch.rand((5, n, 8), dtype=torch.float64, device="cuda", generator=g) * 2.2 - 1.1 for _ in range(8)]
    for t in range(5):
        env.step(acts[t % 8])
    torch.cuda.synchronize()
    F = env._fused
    t0 = time.perf_counter()
    solved = 0
    for t in range(steps):
        env.step(acts[t % 8])
        torch.cuda.synchronize()
        solved += int(F["od_count"][F["bufs"].od_parity & 1])
    dt = (time.perf_counter() - t0) / steps
    return dt * 1e6, solved / steps


for every in (0, 1):
    us, sv = run(every)
    extra = " -> %.2f us per solve (64 per wave, sequential)" % (us / 64) if every else ""
    print("every=%d: %.1f us per step (synchronized), %.0f envs solved per step%s" % (every, us, sv, extra))
