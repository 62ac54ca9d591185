"""Host cost of the Home-Steward step at a tiny batch (GPU far ahead): the whole
env.step, the bare pgw_hs_step call, and a cProfile of the step loop."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from powergridworld_amd import _lib
from powergridworld_amd.base_hs import HSMultiComponentEnv
from powergridworld_amd.scenarios.heterogeneous_hs import make_env_config

for n in (256, 65536):
    env = HSMultiComponentEnv(**make_env_config(), num_envs=n, device=torch.device("cuda", 0))
    act = torch.zeros((n, len(env.envs)), dtype=torch.float64, device="cuda")
    env.reset()

    def run(k):
        for _ in range(k):
            _, _, d, _ = env.step(act)
            if d:
                env.reset()
    run(300)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(572)
    torch.cuda.synchronize()
    print("n=%d env.step: %.1f us/step" % (n, (time.perf_counter() - t0) / 572 * 1e6))
pr = cProfile.Profile()
pr.enable()
run(572)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(12)
