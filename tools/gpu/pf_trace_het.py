"""Phase timeline of k_pf_solve waves (debug trace) in the heterogeneous
scenario's step (all output rows, min/max epilogue) at N = 65536."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tools"))
from powergridworld_amd import _lib
from powergridworld_amd.multiagent_env import MultiAgentEnv
from powergridworld_amd.scenarios.heterogeneous import make_env_config

n = 65536
dev = torch.device("cuda", 0)
env = MultiAgentEnv(**make_env_config(), num_envs=n, device=dev)
gen = torch.Generator(dev).manual_seed(0)


def acts():
    return {a.name: ({c.name: torch.empty((n, c.action_space.shape[0]), dtype=torch.float64,
                                           device=dev).uniform_(-1, 1, generator=gen) for c in a.envs}
                     if hasattr(a, "envs") else
                     torch.empty((n, a.action_space.shape[0]), dtype=torch.float64,
                                 device=dev).uniform_(-1, 1, generator=gen))
            for a in env.agents}


env.reset()
for _ in range(40):
    env.step(acts())
torch.cuda.synchronize()
buf = torch.zeros((4 * n // 64, 8), dtype=torch.int64, device="cuda")   # headroom for table solves
_lib.check(_lib.lib().pgw_debug_pf_trace(_lib.dptr(buf)))
names = ["start", "load+powers", "initial", "iterate", "v0+sig+sync", "rows"]
for rep in range(3):
    a = acts()
    torch.cuda.synchronize()
    buf.zero_()
    env.step(a)
    torch.cuda.synchronize()
    t = buf[: n // 64].cpu().numpy().astype(np.float64) / 100.0      # us
    t0 = t[:, 0].min()
    print("step %d: waves start spread %.2f us, end spread %.2f us, kernel span %.2f us" %
          (rep, t[:, 0].max() - t0, t[:, 5].max() - t[:, 5].min(), t[:, 5].max() - t0))
    for k in range(1, 6):
        d = t[:, k] - t[:, k - 1]
        print("   %-12s mean %6.2f  p50 %6.2f  p99 %6.2f  max %6.2f us" %
              (names[k], d.mean(), np.median(d), np.percentile(d, 99), d.max()))
    it = env.pf_solver.iterations.view(-1, 64)
    print("   iterations: mean %.2f, wave max mean %.2f" % (it.double().mean().item(),
                                                          it.max(1).values.double().mean().item()))
_lib.check(_lib.lib().pgw_debug_pf_trace(None))
