"""Mean PF iterations and solve time, cold start vs warm start (OpenDSSSolver
warm_start), two controllable buses (no predictor table), 65 536 envs."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from powergridworld_amd.distribution_system.opendss import OpenDSSSolver  # noqa: E402

n, dev = 65536, torch.device("cuda", 0)
kw = dict(feeder_file="ieee_13_dss/IEEE13Nodeckt.dss", loadshape_file="ieee_13_dss/annual_hourly_load_profile.csv",
          system_load_rescale_factor=0.7, num_envs=n, device=dev)
rng = np.random.default_rng(21)
base = torch.tensor(rng.uniform(0, 400, size=(2, n)), device=dev)
steps = [base + torch.tensor(rng.normal(0, 15, size=(2, n)), device=dev) for _ in range(60)]
for name, warm in (("cold", False), ("warm", True)):
    s = OpenDSSSolver(**kw, warm_start=warm)
    its = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t, p in enumerate(steps):
        s.calculate_power_flow(p_controllable_consumed={"675c": p[0], "671": p[1]},
                               current_time="2020-08-12 %02d:%02d:00" % (t // 12, 5 * (t % 12)))
        its.append(s.iterations.clone())
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / len(steps) * 1e6
    m = [float(i.double().mean()) for i in its]
    print("%s: mean iterations %.2f (first %.2f, rest %.2f), %.1f us per solve (all 41 rows)"
          % (name, np.mean(m), m[0], np.mean(m[1:]), dt), flush=True)
