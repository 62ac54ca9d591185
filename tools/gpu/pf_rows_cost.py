"""Cost of the output rows of k_pf_solve at N = 65536 (HET's solve: 41 rows,
min / max epilogue): every row stored, vs extrema only (v_out = NULL), vs one
row.  Library events (pgw_timing) around the launches."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from powergridworld_amd import _lib
from powergridworld_amd.distribution_system.opendss import OpenDSSSolver

n = 65536
dev = torch.device("cuda", 0)
pf = OpenDSSSolver("ieee_13_dss/IEEE13Nodeckt.dss", "ieee_13_dss/annual_hourly_load_profile.csv",
                   system_load_rescale_factor=0.65, num_envs=n, device=dev)
p675 = torch.empty(n, dtype=torch.float64, device=dev).uniform_(-400, 200)
ts = "2020-08-12 10:00"
pf.calculate_power_flow({"675c": p675}, None, current_time=ts)       # tables for the hour
torch.cuda.synchronize()
lib = _lib.lib()
p = pf.step_params(ts)
t = pf.step_tables(ts)
cp = p675.reshape(1, n)
vmin = torch.empty(n, dtype=torch.float64, device=dev)
vmax = torch.empty_like(vmin)
t2 = _lib.PFTables.from_buffer_copy(t)
t2.v_min_out, t2.v_max_out = vmin.data_ptr(), vmax.data_ptr()
st = _lib.stream_ptr(dev)


def run(params, tables, v_out, label, reps=200):
    for _ in range(20):
        _lib.check(lib.pgw_pf_solve(params, tables, n, cp.data_ptr(), None, v_out, None, st))
    torch.cuda.synchronize()
    _lib.check(lib.pgw_timing_start(1))
    for _ in range(reps):
        _lib.check(lib.pgw_pf_solve(params, tables, n, cp.data_ptr(), None, v_out, None, st))
    torch.cuda.synchronize()
    ms, cnt = (ctypes.c_double * 8)(), (ctypes.c_int64 * 8)()
    _lib.check(lib.pgw_timing_stop(ms, cnt))
    k = 2                                        # PGW_T_PF_SOLVE
    print("%-34s %7.2f us/launch (%d timed)" % (label, ms[k] * 1e3 / max(cnt[k], 1), cnt[k]))


print("n_out =", p.n_out)
run(p, t2, pf.v_out.data_ptr(), "all rows stored + extrema")
run(p, t2, None, "extrema only (v_out NULL)")
p1 = _lib.PFParams.from_buffer_copy(p)
p1.n_out = 1
run(p1, t, pf.v_out.data_ptr(), "one row (n_out = 1)")
