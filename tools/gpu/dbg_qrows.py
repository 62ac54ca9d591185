"""Debug: HET fused step with row records on / off; on a vmin mismatch print
the env, its bus kW, both values and the value of a full solve (od_table=False)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from powergridworld_amd.multiagent_env import MultiAgentEnv  # noqa
from powergridworld_amd.scenarios.heterogeneous import make_env_config  # noqa
from powergridworld_amd.distribution_system.opendss import OpenDSSSolver  # noqa

DEV = "cuda:0"
n = 8192
envs = [MultiAgentEnv(**make_env_config(), num_envs=n, device=DEV, fused=True) for _ in range(4)]
envs[1].pf_solver.od_row_records = False
envs[2].pf_solver.od_row_records = False
envs[2].pf_solver.od_row_masks = False
envs[3].pf_solver.od_row_masks = False
for e_ in envs[1:]:
    e_.pf_solver._tables_cache.clear()
for env in envs:
    for k, ag in enumerate(env.agents):
        for c in (ag.envs if hasattr(ag, "envs") else [ag]):
            if hasattr(c, "seed"):
                c.seed(70 + k)
    env.reset()
s0 = envs[0].pf_solver
print("qinfo", {k: v for k, v in s0._od_qinfo.items() if v is not None})
print("output names", len(s0.output_names), s0.output_names[:5])
rng = np.random.default_rng(31)
for t in range(30):
    a = torch.tensor(rng.uniform(-1.1, 1.1, (n, 10)), device=DEV)
    act = {"building": {"building": a[:, :6], "pv": a[:, 6:7], "storage": a[:, 7:8]},
           "pv": a[:, 8:9], "ev-charging": a[:, 9:10]}
    out = []
    for env in envs:
        env.step(act)
        vmin, vmax = env.pf_solver.voltage_extrema()
        out.append((vmin.clone(), vmax.clone(), env.pf_solver.iterations.clone(), env._ma["bus_p"][0].clone()))
    (a0, b0, i0, p0), (a1, b1, i1, p1), (a2, b2, i2, p2), (a3, b3, i3, p3) = out
    bad = ((a0 - a1).abs() / a1 > 1e-12) | ((b0 - b1).abs() / b1 > 1e-12)
    if bad.any():
        idx = bad.nonzero().flatten()[:5]
        print("step", t, "time", envs[0].time, "hour", s0.hour_of(envs[0].time), "bad envs", int(bad.sum()))
        full = OpenDSSSolver(**dict(envs[0].pf_config["config"], od_table=False), num_envs=len(idx), device=DEV)
        full.set_controllable_loads(s0._ctrl_names)
        full.calculate_power_flow({s0._ctrl_names[0]: p0[idx]}, current_time=envs[0].time)
        bv = full.get_bus_voltages()
        st = torch.stack(list(bv.values()))
        for j, e in enumerate(idx.tolist()):
            print("  P per env", [float(x[e]) for x in (p0, p1, p2, p3)])
            print("  env %d P %.9f it %d/%d vmin q %.15f noq %.15f nomask %.15f q-nomask %.15f (full %.15f)" % (
                e, p0[e].item(), i0[e].item(), i1[e].item(), a0[e].item(), a1[e].item(), a2[e].item(), a3[e].item(),
                st[:, j].min().item()))
        break
else:
    print("no mismatch in 30 steps")
