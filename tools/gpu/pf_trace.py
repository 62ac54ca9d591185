"""Phase timeline of k_coord_pf waves (debug trace): per-phase durations across
the waves of one C4 step at N = 65536, and the waves' start/end spread."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from powergridworld_amd import _lib
from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config

n = 65536
env = CoordinatedMultiBuildingControlEnv(**make_c4_config(), num_envs=n, device=torch.device("cuda", 0),
                                         fused=True)
gen = torch.Generator("cuda").manual_seed(0)
env.reset()
for _ in range(40):
    env.step(torch.empty((5, n, 8), dtype=torch.float64, device="cuda").uniform_(-1, 1, generator=gen))
torch.cuda.synchronize()
split = os.environ.get("PGW_PF_SPLIT", "0").startswith("1")
half = os.environ.get("PGW_PF_HALF", "0").startswith("1")
# envs per PF wave (k_coord_pf_split: two lanes per env; k_coord_pf with half
# waves: 32 envs, each on two lanes) -- the buffer needs 8 slots per wave
wenv = 32 if (split or half) else 64
print("kernel:", "k_coord_pf_split" if split else "k_coord_pf", "envs per wave", wenv)
buf = torch.zeros((n // wenv, 8), dtype=torch.int64, device="cuda")
_lib.check(_lib.lib().pgw_debug_pf_trace(_lib.dptr(buf)))
for rep in range(3):
    env.step(torch.empty((5, n, 8), dtype=torch.float64, device="cuda").uniform_(-1, 1, generator=gen))
    torch.cuda.synchronize()
    t = buf.cpu().numpy().astype(np.float64) / 100.0      # us
    t0 = t[:, 0].min()
    names = ["start", "load+powers", "initial", "iterate", "currents", "outputs"]
    print("step %d: waves start spread %.2f us, end spread %.2f us, kernel span %.2f us" %
          (rep, t[:, 0].max() - t0, t[:, 5].max() - t[:, 5].min(), t[:, 5].max() - t0))
    for k in range(1, 6):
        d = t[:, k] - t[:, k - 1]
        print("   %-12s mean %6.2f  p50 %6.2f  p99 %6.2f  max %6.2f us" %
              (names[k], d.mean(), np.median(d), np.percentile(d, 99), d.max()))
    it = env.pf_solver.iterations.view(-1, wenv).max(1).values.cpu().numpy()
    slow = np.argmax(t[:, 5])
    print("   slowest wave %d: iterations %d, phases %s" % (slow, it[slow], np.round(np.diff(t[slow, :6]), 2)))
_lib.check(_lib.lib().pgw_debug_pf_trace(None))
