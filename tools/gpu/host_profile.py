"""Host-side cost of the fused C4 step: wall time per step with the GPU far
ahead (small batch) and a cProfile of the same loop (top functions)."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
env = CoordinatedMultiBuildingControlEnv(**make_c4_config(), num_envs=n, device=torch.device("cuda", 0),
                                         fused=True)
act = torch.zeros((5, n, 8), dtype=torch.float64, device="cuda")


def run(k):
    for _ in range(k):
        _, _, d, _ = env.step(act)
        if d["__all__"]:
            env.reset()


env.reset()
run(300)
torch.cuda.synchronize()
for label in ("episode-2+ (caches warm)",):
    t0 = time.perf_counter()
    run(572)
    torch.cuda.synchronize()
    print("%s: %.1f us/step (batch %d)" % (label, (time.perf_counter() - t0) / 572 * 1e6, n))
env2 = CoordinatedMultiBuildingControlEnv(**make_c4_config(), num_envs=n, device=torch.device("cuda", 0),
                                          fused=True)
env = env2
env.reset()
torch.cuda.synchronize()
t0 = time.perf_counter()
run(286)
torch.cuda.synchronize()
print("first episode (cold caches): %.1f us/step" % ((time.perf_counter() - t0) / 286 * 1e6))
pr = cProfile.Profile()
pr.enable()
run(572)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
