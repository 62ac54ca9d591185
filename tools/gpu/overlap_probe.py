"""C4 at 65,536 envs, fused step synchronous vs overlap_pf=True (PF of step t
beside the agents of step t+1): us/step over a driver-shaped region and the
event-timed kernels.  Usage: python tools/gpu/overlap_probe.py [--steps 200]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from powergridworld_amd import _lib  # noqa: E402
from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config  # noqa

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--n", type=int, default=65536)
ap.add_argument("--modes", default="opendss,exact")
ap.add_argument("--overlap", default="0,1", help="which of sync (0) / overlap (1) to run")
ap.add_argument("--no-timing", action="store_true", help="skip the event-timed pass (under a profiler)")
a = ap.parse_args()
dev = torch.device("cuda:0")
n = a.n
gen = torch.Generator(dev).manual_seed(0)
pool = torch.empty((16, 5, 8, n), dtype=torch.float64, device=dev).uniform_(-1, 1, generator=gen).transpose(2, 3)
for conv in a.modes.split(","):
    for ov in [bool(int(x)) for x in a.overlap.split(",")]:
        env = CoordinatedMultiBuildingControlEnv(**make_c4_config(pf_convergence=conv), num_envs=n, device=dev,
                                                 fused=True, overlap_pf=ov)
        env.reset()
        k = [0]

        def run(m):
            for _ in range(m):
                _, _, d, _ = env.step(pool[k[0] % 16])
                k[0] += 1
                if d["__all__"]:
                    env.reset()
        run(30)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(a.steps)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / a.steps * 1e6
        ks = {}
        if not a.no_timing:
            _lib.check(_lib.lib().pgw_timing_start(1))
            run(64)
            torch.cuda.synchronize()
            tot = (_lib.C.c_double * 6)()
            cnt = (_lib.C.c_int64 * 6)()
            _lib.check(_lib.lib().pgw_timing_stop(tot, cnt))
            ks = {nm: round(tot[i] / cnt[i] * 1e3, 2) for i, nm in enumerate(("agents", "coord_pf", "pf_solve"))
                  if cnt[i]}
        print("%-8s overlap=%d  %7.2f us/step  kernels %s" % (conv, ov, us, ks), flush=True)
        del env
        torch.cuda.synchronize()
