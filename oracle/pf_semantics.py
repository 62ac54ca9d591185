"""How far is the exact PF fixed point from what OpenDSS would report?
(TEST INFRASTRUCTURE: oracle only; writes profiles/r03/pf_semantics.txt.)

The reference's voltages come from OpenDSS's ``Solve mode=snap``
(opendss.py:134), which stops its current-injection iteration at a 1e-4
per-unit magnitude change (at least 2, at most 15 iterations).  This script
replays C4 and heterogeneous-scenario load streams through both
``Feeder.solve`` (the exact fixed point at 1e-10, the engine's default) and
``Feeder.snap_opendss`` (OpenDSS's stopped iterate, under both readings of
which load admittances sit in Y), and reports the maxima of the differences in
V675.3, voltage violation, coordinated reward, min voltage and every node.

Usage:  python oracle/pf_semantics.py [--k 256] [--out profiles/r03/pf_semantics.txt]
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)

from oracle.ma_oracle import CoordinatedOracle  # noqa: E402
from oracle.pf_oracle import BatchedPF  # noqa: E402


class RecordingPF(BatchedPF):
    """BatchedPF that records every call's per-load kW / kvar."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.calls = []

    def calculate(self, current_time, p_ctrl=None, q_ctrl=None, K=1):
        self.calls.append(self.loads(current_time, p_ctrl, q_ctrl, K))
        return super().calculate(current_time, p_ctrl, q_ctrl, K)


def c4_streams(k_random, seed=0):
    """(kw, kvar) per PF call: the c4_two_episodes golden actions (2 envs x 2
    episodes, the reference's SoC draws) and k_random envs of uniform actions."""
    g = np.load(os.path.join(REPO, "tests", "golden", "c4_two_episodes.npz"))
    out = []
    ora = CoordinatedOracle(K=2)
    ora.pf = RecordingPF(system_load_rescale_factor=1.2)
    for e in range(g["actions"].shape[0]):
        ora.reset(g["init_storage"][e])
        for t in range(g["actions"].shape[1]):
            ora.step(g["actions"][e, t])
    out += ora.pf.calls
    rng = np.random.default_rng(seed)
    ora = CoordinatedOracle(K=k_random)
    ora.pf = RecordingPF(system_load_rescale_factor=1.2)
    ora.reset(rng.uniform(3.0, 50.0, size=(5, k_random)))
    for t in range(286):
        ora.step(rng.uniform(-1, 1, size=(5, k_random, 8)))
    out += ora.pf.calls
    return out


def het_streams(k_random, seed=1):
    """Heterogeneous scenario (scenarios/heterogeneous.py: MC building at 675c,
    PV farm at 675, EV 25x40 at 671; rescale 0.65): bus loads built from
    uniform powers in each agent's physical range, per step."""
    pf = RecordingPF(system_load_rescale_factor=0.65)
    rng = np.random.default_rng(seed)
    import pandas as pd
    t = pd.Timestamp("08-12-2021 00:00:00")
    for s in range(286):
        t = t + pd.Timedelta(300, "s")
        bld = rng.uniform(-20, 160, k_random)          # building + PV + storage net kW
        pv = -rng.uniform(0, 800, k_random)            # PV farm generation
        ev = rng.uniform(0, 300, k_random)             # 25 vehicles x 40 multiplier, kWh/step as kW
        p = {"675c": bld, "675a": pv / 3, "675b": pv / 3, "671": ev}
        pf.calculate(t, p, K=k_random)
    return pf.calls


def compare(calls, feeder, node675, label, lines):
    vmax = {"H2": [], "H1": []}
    stats = {h: dict(dv675=0.0, dv675_rel=0.0, dvv=0.0, drew=0.0, dnode_rel=0.0, dmin=0.0,
                     iters=np.zeros(16, int)) for h in ("H2", "H1")}
    h12 = 0.0
    for kw, kvar in calls:
        Vx, _ = feeder.solve(kw, kvar, tol=1e-10)
        px = feeder.pu(Vx)
        res = {}
        for h in ("H2", "H1"):
            if h == "H2":
                V, it = feeder.snap_opendss(kw, kvar, feeder.base_kw, feeder.base_kvar)
            else:
                V, it = feeder.snap_opendss(kw, kvar)
            p = feeder.pu(V)
            res[h] = p
            st = stats[h]
            d675 = np.abs(p[:, node675] - px[:, node675])
            st["dv675"] = max(st["dv675"], d675.max())
            st["dv675_rel"] = max(st["dv675_rel"], (d675 / px[:, node675]).max())
            vv = lambda v: np.maximum(np.maximum(0.0, 0.95 - v), v - 1.05)
            dvv = np.abs(vv(p[:, node675]) - vv(px[:, node675]))
            st["dvv"] = max(st["dvv"], dvv.max())
            st["drew"] = max(st["drew"], (dvv * 1e4 / 5).max())
            st["dnode_rel"] = max(st["dnode_rel"], (np.abs(p - px) / px).max())
            st["dmin"] = max(st["dmin"], np.abs(p.min(1) - px.min(1)).max())
            np.add.at(st["iters"], it, 1)
        h12 = max(h12, (np.abs(res["H1"] - res["H2"]) / px).max())
    n = sum(c[0].shape[0] for c in calls)
    lines.append("%s: %d solves" % (label, n))
    for h, st in stats.items():
        name = ("H2 (Y holds the DSS file's load Yeq; the Loads.kW setter leaves Yprim valid)"
                if h == "H2" else "H1 (Y re-stamped with each step's load Yeq)")
        lines.append("  OpenDSS snap %s vs exact fixed point (1e-10):" % name)
        lines.append("    max |dV675.3|            %.3e pu   (rel %.3e)" % (st["dv675"], st["dv675_rel"]))
        lines.append("    max |d voltage_violation| %.3e" % st["dvv"])
        lines.append("    max |d coordinated reward| %.3e  (1e4 * dvv / 5)" % st["drew"])
        lines.append("    max rel |dV| over all nodes %.3e" % st["dnode_rel"])
        lines.append("    max |d min voltage|      %.3e pu" % st["dmin"])
        its = {i: int(c) for i, c in enumerate(st["iters"]) if c}
        lines.append("    iterations used: %s" % its)
    lines.append("  H1 vs H2, max rel |dV| over all nodes: %.3e" % h12)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=256)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r03", "pf_semantics.txt"))
    a = ap.parse_args()
    pf = BatchedPF(system_load_rescale_factor=1.2)
    f = pf.feeder
    node = f.idx["675.3"]
    lines = ["PF semantics: OpenDSS's stopped snap iterate vs the exact fixed point "
             "(oracle/pf_semantics.py --k %d)" % a.k, ""]
    compare(c4_streams(a.k), f, node, "C4 (c4_two_episodes golden streams + %d uniform-action envs x 286 steps)"
            % a.k, lines)
    lines.append("")
    compare(het_streams(a.k), f, node, "HET-like (uniform agent powers at 675c / 675 / 671, rescale 0.65, "
            "%d envs x 286 steps)" % a.k, lines)
    text = "\n".join(lines) + "\n"
    print(text)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        fh.write(text)


if __name__ == "__main__":
    main()
