"""Host cost of the heterogeneous step on the fused multi-agent path: env.step
at a tiny batch (the GPU never bounds it) and at 65 536 envs, plus a cProfile."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from powergridworld_amd.multiagent_env import MultiAgentEnv  # noqa: E402
from powergridworld_amd.scenarios.heterogeneous import make_env_config  # noqa: E402

dev = torch.device("cuda", 0)
for n in (256, 65536):
    env = MultiAgentEnv(**make_env_config(), num_envs=n, device=dev)
    gen = torch.Generator(dev).manual_seed(0)
    acts = [{a.name: ({c.name: torch.empty((n, c.action_space.shape[0]), dtype=torch.float64, device=dev)
                       .uniform_(-1, 1, generator=gen) for c in a.envs} if hasattr(a, "envs") else
                      torch.empty((n, a.action_space.shape[0]), dtype=torch.float64, device=dev)
                      .uniform_(-1, 1, generator=gen)) for a in env.agents} for _ in range(8)]
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
    run(572)
    torch.cuda.synchronize()
    print("n=%d env.step: %.1f us/step" % (n, (time.perf_counter() - t0) / 572 * 1e6), flush=True)
pr = cProfile.Profile()
pr.enable()
run(572)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(14)
