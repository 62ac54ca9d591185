"""Host cost of the heterogeneous scenario's first episode against a later
one (65,536 envs, fused path): us per step and a cProfile of each, to find the
per-episode-position work done on first use."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from powergridworld_amd.multiagent_env import MultiAgentEnv   # noqa: E402
from powergridworld_amd.scenarios.heterogeneous import make_env_config   # noqa: E402

dev = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
env = MultiAgentEnv(**make_env_config(), num_envs=n, device=dev)
gen = torch.Generator(dev).manual_seed(0)
acts = [{ag.name: ({c.name: torch.empty((n, c.action_space.shape[0]), dtype=torch.float64, device=dev)
                    .uniform_(-1, 1, generator=gen) for c in ag.envs} if hasattr(ag, "envs") else
                   torch.empty((n, ag.action_space.shape[0]), dtype=torch.float64, device=dev)
                   .uniform_(-1, 1, generator=gen)) for ag in env.agents} for _ in range(8)]
env.reset()
k = [0]


def episode():
    for _ in range(286):
        _, _, d, _ = env.step(acts[k[0] % 8])
        k[0] += 1
        if d["__all__"]:
            env.reset()


for ep in range(2):
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pr.enable()
    episode()
    pr.disable()
    torch.cuda.synchronize()
    print("episode %d: %.2f us/step" % (ep, (time.perf_counter() - t0) / 286 * 1e6), flush=True)
    pstats.Stats(pr).sort_stats("tottime").print_stats(14)
