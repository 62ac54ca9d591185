"""Where a driver-shaped timed region (--steps 20) loses its time: the C4 bench
env at 65,536 envs, timed regions of 20 steps repeated under variants, with a
host timestamp after every env.step and after the closing synchronize.

  python tools/gpu/short_region.py [reps]
"""
import gc
import os
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n, K = 65536, 20
dev = torch.device("cuda", 0)
env = CoordinatedMultiBuildingControlEnv(**make_c4_config(), num_envs=n, device=dev, fused=True)
gen = torch.Generator(dev).manual_seed(0)
pool = torch.empty((64, 5, 8, n), dtype=torch.float64, device=dev)
pool.uniform_(-1.0, 1.0, generator=gen)
packed = pool.transpose(2, 3)
env.reset()
k = [0]


def run(m, ts=None):
    for _ in range(m):
        _, _, d, _ = env.step(packed[k[0] % 64])
        k[0] += 1
        if d["__all__"]:
            env.reset()
        if ts is not None:
            ts.append(time.perf_counter())


def region(label, pre=None, spin_us=0):
    if pre:
        pre()
    torch.cuda.synchronize()
    if spin_us:
        t = time.perf_counter()
        while time.perf_counter() - t < spin_us * 1e-6:
            pass
    ts = []
    t0 = time.perf_counter()
    run(K, ts)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    host = [round((x - t0) * 1e6, 1) for x in ts]
    print("%-28s %.2f us/step | host issue %.0f us, sync wait %.0f us | first steps %s | last %s"
          % (label, (t2 - t0) / K * 1e6, (t1 - t0) * 1e6, (t2 - t1) * 1e6, host[:4], host[-2:]))


run(30)
for r in range(reps):
    region("plain")
    region("after gc.collect", pre=gc.collect)
    region("gc.collect + 5 steps", pre=lambda: (gc.collect(), run(5)))
    region("idle 50 ms", pre=lambda: time.sleep(0.05))
    region("idle 50 ms + 5 steps", pre=lambda: (time.sleep(0.05), run(5)))
    region("spin 100 us after sync", spin_us=100)
# steady state of a long region for comparison
torch.cuda.synchronize()
t0 = time.perf_counter()
run(572)
torch.cuda.synchronize()
print("572-step region %.2f us/step" % ((time.perf_counter() - t0) / 572 * 1e6))
