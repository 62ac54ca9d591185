"""Phase timeline of k_coord_pf_od waves (the C4 headline PF, OpenDSS rule with
its response table) from the debug trace (pgw_debug_pf_trace: the trace
instantiation stamps wall_clock64(), 100 MHz): per phase the waves' durations,
the waves' start / end spread, the kernel span.  N = 65 536, fused C4 step.
Usage: python tools/gpu/pf_od_trace.py [--steps 6]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from powergridworld_amd import _lib  # noqa: E402
from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config  # noqa

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=6)
a = ap.parse_args()
n = 65536
dev = torch.device("cuda", 0)
env = CoordinatedMultiBuildingControlEnv(**make_c4_config(), num_envs=n, device=dev, fused=True)
gen = torch.Generator(dev).manual_seed(0)
env.reset()
act = lambda: torch.empty((5, n, 8), dtype=torch.float64, device=dev).uniform_(-1, 1, generator=gen)
for _ in range(40):
    env.step(act())
torch.cuda.synchronize()
buf = torch.zeros((n // 64, 8), dtype=torch.int64, device=dev)
names = ["entry", "powers", "lookup", "fallback", "node0", "rows", "atomics"]
_lib.check(_lib.lib().pgw_debug_pf_trace(_lib.dptr(buf)))
try:
    for rep in range(a.steps):
        buf.zero_()
        env.step(act())
        torch.cuda.synchronize()
        t = buf.cpu().numpy().astype(np.float64) / 100.0      # us
        t0 = t[:, 0].min()
        print("step %d: waves' start spread %.2f us, end spread %.2f us, kernel span %.2f us" %
              (rep, t[:, 0].max() - t0, t[:, 6].max() - t[:, 6].min(), t[:, 6].max() - t0), flush=True)
        for k in range(1, 7):
            d = t[:, k] - t[:, k - 1]
            print("   %-9s mean %6.2f  p50 %6.2f  p99 %6.2f  max %6.2f us" %
                  (names[k], d.mean(), np.median(d), np.percentile(d, 99), d.max()), flush=True)
finally:
    _lib.check(_lib.lib().pgw_debug_pf_trace(None))
