"""Host time of each env.step call (no sync) over the first steps of a fresh C4
env at the bench batch -- the driver's short bench (--warmup 5 --steps 20) runs
exactly these steps -- and a cProfile of steps 5..25."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
dev = torch.device("cuda", 0)
pool = torch.rand((64, 5, 8, n), dtype=torch.float64, device=dev) * 2 - 1
packed = pool.transpose(2, 3)
for rep in range(2):
    t0 = time.perf_counter()
    env = CoordinatedMultiBuildingControlEnv(**make_c4_config(), num_envs=n, device=dev, fused=True)
    t1 = time.perf_counter()
    env.reset()
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    print("construct %.1f ms, reset %.1f ms (host), sync %.1f ms" % ((t1 - t0) * 1e3, (t2 - t1) * 1e3,
                                                                    (time.perf_counter() - t2) * 1e3))
    ts = []
    pr = cProfile.Profile()
    for k in range(30):
        if k == 5 and rep == 1:
            pr.enable()
        a = time.perf_counter()
        env.step(packed[k % 64])
        ts.append((time.perf_counter() - a) * 1e6)
    pr.disable()
    torch.cuda.synchronize()
    print("rep %d host us per step:" % rep, [round(x, 1) for x in ts])
    if rep == 1:
        pstats.Stats(pr).sort_stats("tottime").print_stats(20)
    # steady state: second episode
    for k in range(30, 286 + 30):
        _, _, d, _ = env.step(packed[k % 64])
        if d["__all__"]:
            env.reset()
    torch.cuda.synchronize()
    ts = []
    for k in range(30):
        a = time.perf_counter()
        env.step(packed[k % 64])
        ts.append((time.perf_counter() - a) * 1e6)
    torch.cuda.synchronize()
    print("warm host us per step:", [round(x, 1) for x in ts])
