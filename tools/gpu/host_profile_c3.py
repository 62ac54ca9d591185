"""Host cost of the C3 MultiComponentEnv step (building + PV + storage + EV(100))
at a small batch, where the GPU never bounds the step: mean host time per
env.step and a cProfile of 572 steps (the bench's action pool of 16)."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tools"))
from bench_configs import c3_env   # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
dev = torch.device("cuda", 0)
env, acts = c3_env(dev, n)
env.reset()
k = [0]


def run(m):
    for _ in range(m):
        _, _, d, _ = env.step(acts[k[0] % len(acts)])
        k[0] += 1
        if d:
            env.reset()


run(300)
torch.cuda.synchronize()
for _ in range(3):
    t0 = time.perf_counter()
    run(572)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print("host %.2f us/step, with sync %.2f us/step" % ((t1 - t0) / 572 * 1e6, (time.perf_counter() - t0) / 572 * 1e6))
pr = cProfile.Profile()
pr.enable()
run(572)
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
