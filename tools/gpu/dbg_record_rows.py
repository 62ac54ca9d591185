"""Debug: per-record candidate slots of the heterogeneous scenario's row
records (OpenDSSSolver._od_qrows) -- how many slots each record keeps, which
rows, and how the count moves with the bound's samples / delta."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from powergridworld_amd.multiagent_env import MultiAgentEnv  # noqa
from powergridworld_amd.scenarios.heterogeneous import make_env_config  # noqa
from powergridworld_amd.distribution_system import opendss as od  # noqa

env = MultiAgentEnv(**make_env_config(), num_envs=256, device="cuda:0", fused=True)
env.reset()
s = env.pf_solver
names = list(s.output_names)
for key, info in list(s._od_qinfo.items())[:3]:
    if info is None:
        continue
    idx = key[0]
    rows = [r for r in range(64) if (info[0] >> r) & 1]
    print("table row", idx, "slots", [names[r] for r in rows])
    q = s._od_qrec[idx]
    recs = s._od_resp[idx]
    meta = recs.view(torch.int64)[:, 4]
    live = ((meta & 0xffffffff) != 0) & (recs[:, 0] <= recs[:, 1])
    bits = q.view(torch.int64)[:, 5][live].cpu().numpy()
    cnt = np.array([bin(int(b) & ((1 << 64) - 1)).count("1") for b in bits])
    print("  live records", len(bits), "candidate slots per record: mean %.2f hist %s" % (
        cnt.mean(), np.bincount(cnt).tolist()))
    per_slot = [(names[rows[k]], int(((bits >> k) & 1).sum())) for k in range(len(rows))]
    print("  records per slot", per_slot)
    # the same with tighter bounds
    f, M, dev = s.feeder, s.M, s.device
    vrow = names.index(f.node_names[s._od_vnode()]) if s._od_vnode() is not None else -1
    cmp = rows + ([vrow] if vrow > 0 else [])
    nodes = [f.node_index[names[r]] for r in cmp]
    G = torch.from_numpy(np.ascontiguousarray(s._od_Gall[nodes][:, :M])).to(dev)
    V0 = torch.from_numpy(np.ascontiguousarray(s._od_V0all[nodes])).to(dev)
    rl = recs[live]
    c = torch.view_as_complex(rl[:, 6:6 + 6 * M].reshape(-1, 3, M, 2).contiguous())
    abc = torch.einsum("pqm,rm->pqr", c, G)
    tl, th = (rl[:, 0] - rl[:, 2]) * rl[:, 3], (rl[:, 1] - rl[:, 2]) * rl[:, 3]
    for S_, d in ((9, 1e-9), (33, 1e-9), (33, 1e-10), (129, 1e-11)):
        cand = od.extrema_candidates_per_piece(abc[:, 0] + V0, abc[:, 1], abc[:, 2], tl, th, S_, d)[:, :len(rows)]
        print("  samples %d delta %g: mean slots %.2f" % (S_, d, cand.sum(1).double().mean().item()))
