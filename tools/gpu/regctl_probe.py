"""Probe: cost of RegControl on the general power flow at 65,536 envs
(tests/data/regctl_feeder.dss): calculate_power_flow wall time per call and
control passes, with the RegControls active vs the same feeder with
Controlmode=OFF (fixed DSS taps), and the k_pf_general events of each."""
import ctypes
import os
import sys
import time

import numpy as np
import pandas as pd
import torch

ROOT = os.environ.get("GRAFT_REPO_ROOT", ".")
sys.path.insert(0, ROOT)
from powergridworld_amd import _lib  # noqa: E402
from powergridworld_amd.distribution_system.opendss import OpenDSSSolver  # noqa: E402

N = 65536
dev = torch.device("cuda", 0)
src = os.path.join(ROOT, "tests", "data", "regctl_feeder.dss")
off = os.path.join(ROOT, "gpurun_out", "regctl_off.dss")
os.makedirs(os.path.dirname(off), exist_ok=True)
with open(src) as f:
    text = f.read()
with open(off, "w") as f:
    f.write(text.replace("calcv", "Set Controlmode=OFF\ncalcv"))
lib = _lib.lib()
rng = np.random.default_rng(0)
loads = [torch.tensor(rng.uniform(-300, 900, N), device=dev) for _ in range(8)]
times = [pd.Timestamp("08-12-2021 %02d:00:00" % h) for h in range(24)]
for label, path, warm in (("RegControl", src, False), ("RegControl, warm_start", src, True),
                          ("fixed taps", off, False)):
    s = OpenDSSSolver(path, "ieee_13_dss/annual_hourly_load_profile.csv", num_envs=N, device=dev,
                      warm_start=warm)
    for k in range(4):
        s.calculate_power_flow({"f1": loads[k % 8]}, None, current_time=times[k])
    torch.cuda.synchronize()
    _lib.check(lib.pgw_timing_start(1))
    t0 = time.perf_counter()
    passes = []
    for k in range(16):
        s.calculate_power_flow({"f1": loads[k % 8]}, None, current_time=times[(k + 4) % 24])
        passes.append(getattr(s, "control_iterations", 1))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 16
    tot, cnt = (ctypes.c_double * 8)(), (ctypes.c_int64 * 8)()
    _lib.check(lib.pgw_timing_stop(tot, cnt))
    it = s.iterations.float().abs().mean().item()
    print("%-22s: %.1f us per calculate_power_flow, control passes %s, k_pf_general %.1f us x %d launches, "
          "mean PF iterations (last solve) %.2f" % (label, dt * 1e6, sorted(set(passes)), tot[5] / max(cnt[5], 1) * 1e3,
                                                  cnt[5], it), flush=True)
