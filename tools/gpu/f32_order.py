"""Debug: bench.py's fp32-storage variant alone, then after the graph8 variant
(the order bench.py runs them in), to see which leaves it slow."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa
from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config  # noqa

dev = torch.device("cuda", 0)
n, P = 65536, 64
pick = lambda d: {k: d[k] for k in ("ms_per_step", "k_coord_pf_avg_us") if k in d}
print("f32 alone", json.dumps(pick(bench.f32_variant("opendss", n, 20, 5, P, 1, dev))))
print("f32 alone again", json.dumps(pick(bench.f32_variant("opendss", n, 20, 5, P, 1, dev))))
env = CoordinatedMultiBuildingControlEnv(**make_c4_config(), num_envs=n, device=dev)
pool = torch.rand((P, 5, 8, n), dtype=torch.float64, device=dev) * 2 - 1
packed = pool.transpose(2, 3)
env.reset()
for k in range(30):
    env.step(packed[k % P])
g = bench.graph_variant(env, packed, 20)
print("graph8", g["ms_per_step"])
print("f32 after graph8", json.dumps(pick(bench.f32_variant("opendss", n, 20, 5, P, 1, dev))))
print("f32 after graph8 again", json.dumps(pick(bench.f32_variant("opendss", n, 20, 5, P, 1, dev))))
