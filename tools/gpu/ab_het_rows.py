"""Same-box A/B of the extrema row masks (pgw_pf_od.resp_rows) on the
heterogeneous scenario at 65,536 envs: two envs, one with
OpenDSSSolver.od_row_masks off, stepped alternately in timed regions;
µs per step and the PF kernel's HIP-event average.
Usage: python tools/gpu/ab_het_rows.py [rounds]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from powergridworld_amd import _lib   # noqa: E402
from powergridworld_amd.multiagent_env import MultiAgentEnv   # noqa: E402
from powergridworld_amd.scenarios.heterogeneous import make_env_config   # noqa: E402

dev = torch.device("cuda", 0)
n = 65536
envs = [MultiAgentEnv(**make_env_config(), num_envs=n, device=dev) for _ in range(2)]
envs[1].pf_solver.od_row_masks = False
gen = torch.Generator(dev).manual_seed(0)
acts = []
for _ in range(8):
    acts.append({ag.name: ({c.name: torch.empty((n, c.action_space.shape[0]), dtype=torch.float64,
                                                 device=dev).uniform_(-1, 1, generator=gen) for c in ag.envs}
                           if hasattr(ag, "envs") else
                           torch.empty((n, ag.action_space.shape[0]), dtype=torch.float64,
                                       device=dev).uniform_(-1, 1, generator=gen))
                 for ag in envs[0].agents})
ks = [0, 0]


def run(i, m):
    e = envs[i]
    for _ in range(m):
        _, _, d, _ = e.step(acts[ks[i] % 8])
        ks[i] += 1
        if d["__all__"]:
            e.reset()


for i in range(2):
    envs[i].reset()
    run(i, 300)
m0 = envs[0].pf_solver._od_rowmask
print("masks: rows per hour", sorted(set(bin(m).count("1") for m in m0.values())), "of",
      len(envs[0].pf_solver.output_names), flush=True)
lib = _lib.lib()
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    for i in range(2):
        torch.cuda.synchronize()
        _lib.check(lib.pgw_timing_start(1))
        t0 = time.perf_counter()
        run(i, 286)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 286 * 1e6
        tot = (_lib.C.c_double * 6)()
        cnt = (_lib.C.c_int64 * 6)()
        _lib.check(lib.pgw_timing_stop(tot, cnt))
        pf = tot[2] / max(cnt[2], 1) * 1e3
        ma = tot[4] / max(cnt[4], 1) * 1e3
        print("round %d masks=%d  %.2f us/step (timed launches)  k_ma_step %.2f  PF %.2f" % (r, 1 - i, dt, ma, pf),
              flush=True)
