"""Debug: extrema-only solves (v_out = None) of the HET feeder over a dense kW
sweep in one hour, with row records on, row records off (masked rows) and
masks off; every value checked against the all-rows solve (v_out written)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from powergridworld_amd import _lib  # noqa
from powergridworld_amd.multiagent_env import MultiAgentEnv  # noqa
from powergridworld_amd.scenarios.heterogeneous import make_env_config  # noqa
from powergridworld_amd.distribution_system.opendss import OpenDSSSolver  # noqa

DEV = "cuda:0"
TIME = sys.argv[1] if len(sys.argv) > 1 else "2020-08-12 02:25:00"
cfg = make_env_config()
ctrl = MultiAgentEnv(**cfg, num_envs=64, device=DEV, fused=True).pf_solver._ctrl_names
n = 1 << 20
P = torch.linspace(-900.0, 300.0, n, dtype=torch.float64, device=DEV)
P[:4096] = -283.422709126 + torch.linspace(-0.05, 0.05, 4096, dtype=torch.float64, device=DEV)


def solver(rec, masks, recrows=True):
    s = OpenDSSSolver(**dict(cfg["pf_config"]["config"]), num_envs=n, device=DEV)
    s.set_controllable_loads(ctrl)
    s.od_row_records = rec
    s.od_row_masks = masks
    s.od_record_rows = recrows
    s._tables_cache.clear()
    s._od_qinfo.clear()
    return s


def extrema(s):
    s.calculate_power_flow({ctrl[0]: P}, current_time=TIME)      # builds the hour's tables
    p = s.step_params(TIME)
    t = s.solve_tables(TIME, True)
    it = torch.empty(n, dtype=torch.int32, device=DEV)
    fn = _lib.lib().pgw_pf_solve_general if s.general else _lib.lib().pgw_pf_solve
    _lib.check(fn(p, t, n, P.data_ptr(), None, None, it.data_ptr(), _lib.stream_ptr(DEV)))
    torch.cuda.synchronize()
    return s._vmin.clone(), s._vmax.clone(), it


full = solver(False, False)
full.calculate_power_flow({ctrl[0]: P}, current_time=TIME)
V = full.v_out[:len(full.output_names)].clone()
vmin_f, vmax_f = V.min(0).values, V.max(0).values
rowmin = V.argmin(0)
print("hour", full.hour_of(TIME), "rows", len(full.output_names))
res = {}
for name, (rec, masks, rr) in {"q": (True, True, True), "q-all-slots": (True, True, False),
                               "noq": (False, True, True), "nomask": (False, False, True)}.items():
    s = solver(rec, masks, rr)
    a, b, it = extrema(s)
    res[name] = (a, b)
    idx = s._od_index.get(s.hour_of(TIME)) if hasattr(s, "_od_index") else None
    bad = ((a - vmin_f).abs() > 1e-12) | ((b - vmax_f).abs() > 1e-12)
    st = s.od_resp_stats
    print(name, "bad", int(bad.sum()), "of", n, "record slots: candidates %s of %s" % (
        st.get("record_rows_candidates"), st.get("record_rows_listed")))
    if bad.any():
        for e in bad.nonzero().flatten()[:6].tolist():
            print("  P %.9f vmin %.15f full %.15f (row %s) vmax %.15f full %.15f it %d" % (
                P[e].item(), a[e].item(), vmin_f[e].item(), full.output_names[int(rowmin[e])], b[e].item(),
                vmax_f[e].item(), it[e].item()))
        keys = [k for k in s._od_rowmask]
        for k in keys:
            m = s._od_rowmask[k]
            print("  mask", k, [full.output_names[r] for r in range(64) if (m >> r) & 1])
print("q == q-all-slots bit for bit:", torch.equal(res["q"][0], res["q-all-slots"][0]) and
      torch.equal(res["q"][1], res["q-all-slots"][1]))
