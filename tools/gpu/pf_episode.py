"""Per-step k_coord_pf span (debug trace) and the slowest wave's iterations over
one C4 episode at N = 65536: how much of the PF average is the iteration tail."""
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
buf = torch.zeros((n // 64, 8), dtype=torch.int64, device="cuda")
env.reset()
_lib.check(_lib.lib().pgw_debug_pf_trace(_lib.dptr(buf)))
spans, maxit, typ = [], [], []
for step in range(286):
    _, _, d, _ = env.step(torch.empty((5, n, 8), dtype=torch.float64, device="cuda").uniform_(-1, 1, generator=gen))
    torch.cuda.synchronize()
    t = buf.cpu().numpy().astype(np.float64) / 100.0
    spans.append(t[:, 5].max() - t[:, 0].min())
    typ.append(np.median(t[:, 5] - t[:, 0]))
    maxit.append(int(env.pf_solver.iterations.max()))
    if d["__all__"]:
        break
_lib.check(_lib.lib().pgw_debug_pf_trace(None))
spans, maxit, typ = np.array(spans), np.array(maxit), np.array(typ)
print("steps", len(spans), "span mean %.2f us, median wave %.2f us" % (spans.mean(), typ.mean()))
for k in sorted(set(maxit)):
    m = maxit == k
    print("  max iterations %d: %3d steps, span mean %.2f us" % (k, m.sum(), spans[m].mean()))
print("by hour (max it):", [int(maxit[h * 12:(h + 1) * 12].max()) for h in range(len(maxit) // 12)])
