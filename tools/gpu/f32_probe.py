"""Host profile of the fp32-storage C4 variant (bench.f32_variant's loop):
per-step wall time over an episode with its reset, cProfile top entries."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config  # noqa

dev = torch.device("cuda", 0)
n = 65536
dt = torch.float32 if "--f64" not in sys.argv else torch.float64
env = CoordinatedMultiBuildingControlEnv(**make_c4_config(), num_envs=n, device=dev, dtype=dt)
pool = torch.rand((8, 5, 8, n), dtype=dt, device=dev) * 2 - 1
packed = pool.transpose(2, 3)
env.reset()
k = [0]


def run(m):
    for _ in range(m):
        _, _, d, _ = env.step(packed[k[0] % 8])
        k[0] += 1
        if d["__all__"]:
            t0 = time.perf_counter()
            env.reset()
            torch.cuda.synchronize()
            print("reset %.3f ms" % ((time.perf_counter() - t0) * 1e3))
run(30)
torch.cuda.synchronize()
t0 = time.perf_counter()
pr = cProfile.Profile()
pr.enable()
run(286)
torch.cuda.synchronize()
pr.disable()
print("us/step %.2f" % ((time.perf_counter() - t0) / 286 * 1e6))
pstats.Stats(pr).sort_stats("cumtime").print_stats(18)
