"""Host cost of the heterogeneous scenario's fused step: wall time per step with
the device synchronised after every step vs not, and a cProfile of 286 steps."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from powergridworld_amd.multiagent_env import MultiAgentEnv  # noqa
from powergridworld_amd.scenarios.heterogeneous import make_env_config  # noqa

dev = torch.device("cuda", 0)
n = 65536
env = MultiAgentEnv(**make_env_config(), num_envs=n, device=dev)
g = torch.Generator(dev).manual_seed(0)
acts = []
for _ in range(8):
    acts.append({a.name: ({c.name: torch.empty((n, c.action_space.shape[0]), dtype=torch.float64, device=dev)
                           .uniform_(-1, 1, generator=g) for c in a.envs} if hasattr(a, "envs") else
                          torch.empty((n, a.action_space.shape[0]), dtype=torch.float64, device=dev)
                          .uniform_(-1, 1, generator=g)) for a in env.agents})
env.reset()
k = [0]


def run(m):
    for _ in range(m):
        _, _, d, _ = env.step(acts[k[0] % 8])
        k[0] += 1
        if d["__all__"]:
            env.reset()
run(300)
torch.cuda.synchronize()
t0 = time.perf_counter()
run(286)
torch.cuda.synchronize()
print("us/step %.2f" % ((time.perf_counter() - t0) / 286 * 1e6))
pr = cProfile.Profile()
pr.enable()
run(286)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(22)
