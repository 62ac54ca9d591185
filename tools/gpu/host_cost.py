"""Host cost per fused C4 step at a small batch (GPU never the bottleneck):
whole env.step, and the pgw_coord_step ctypes call alone."""
import os
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from powergridworld_amd import _lib
from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
env = CoordinatedMultiBuildingControlEnv(**make_c4_config(), num_envs=n, device=torch.device("cuda", 0),
                                         fused=True)
act = torch.zeros((5, n, 8), dtype=torch.float64, device="cuda")
env.reset()
lib = _lib.lib()
orig = lib.pgw_coord_step
acc = [0.0, 0]


def timed(*a):
    t0 = time.perf_counter()
    r = orig(*a)
    acc[0] += time.perf_counter() - t0
    acc[1] += 1
    return r


for timing in (False, True):
    for _ in range(300):
        _, _, d, _ = env.step(act)
        if d["__all__"]:
            env.reset()
    torch.cuda.synchronize()
    if timing:
        _lib.check(lib.pgw_timing_start(4))
    lib.pgw_coord_step = timed
    acc[:] = [0.0, 0]
    t0 = time.perf_counter()
    k = 2000
    for _ in range(k):
        _, _, d, _ = env.step(act)
        if d["__all__"]:
            env.reset()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    lib.pgw_coord_step = orig
    if timing:
        tot = (_lib.C.c_double * 8)()
        cnt = (_lib.C.c_int64 * 8)()
        _lib.check(lib.pgw_timing_stop(tot, cnt))
    print("timing=%s: %.1f us/step total, pgw_coord_step call %.1f us" %
          (timing, dt / k * 1e6, acc[0] / max(acc[1], 1) * 1e6))
