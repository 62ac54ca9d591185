"""Time the REFERENCE's own Python step loop on the C4 scenario in THIS container
(SURVEY 8(d) CPU-baseline protocol): one env per process, k = 1 and k = 8
processes (multiprocessing.Pool), stdout to devnull, a stub PowerFlowSolver
(OpenDSS is absent), synthetic exogenous data.

The reference exists only in the build container, never on the GPU box, so
this writes its numbers to profiles/ref_cpu_loop.json and bench.py reports them
as a labelled row beside its own cpu_baseline (the oracle timed on the GPU
host).  Test/measurement infrastructure only.

Usage:  python tools/ref_cpu_loop.py [--steps 286] [--procs 1 8]
"""
import argparse
import json
import os
import platform
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _one(args):
    seed, steps = args
    os.environ["OMP_NUM_THREADS"] = "1"
    sys.path.insert(0, REPO)
    import contextlib
    import copy
    import io
    import numpy as np
    from oracle import make_golden as mg            # imports the reference (gym stub, patched data)
    from gridworld.distribution_system.powerflow import PowerFlowSolver

    class StubPF(PowerFlowSolver):
        """Constant 1.0 pu at every node (stub PF)."""
        def __init__(self, **kw):
            self.v = {}

        def calculate_power_flow(self, p_controllable_consumed=None, q_controllable_consumed=None,
                                 current_time=None):
            self.v = {"675.3": 1.0}

        def get_bus_voltages(self):
            return self.v

        def get_bus_voltage_by_name(self, name):
            return 1.0

    cfg = mg._c4_cfg()
    cfg["pf_config"] = {"cls": StubPF, "config": {}}
    env = mg.CoordinatedEnv(**copy.deepcopy(cfg))
    rng = np.random.default_rng(seed)
    names = [a.name for a in env.agents]
    acts = rng.uniform(-1, 1, (steps, len(names), 8))
    sink = io.StringIO()
    with contextlib.redirect_stdout(sink):
        env.reset()
        t0 = time.perf_counter()
        n = 0
        for t in range(steps):
            _, _, d, _ = env.step({nm: {"building": acts[t, a, :6], "pv": acts[t, a, 6:7],
                                        "storage": acts[t, a, 7:8]} for a, nm in enumerate(names)})
            n += 1
            if d["__all__"]:
                env.reset()
        dt = time.perf_counter() - t0
    return len(names) * n, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=286)
    ap.add_argument("--procs", type=int, nargs="+", default=[1, 8])
    args = ap.parse_args()
    import multiprocessing as mp
    rows = []
    for k in args.procs:
        t0 = time.perf_counter()
        with mp.get_context("fork").Pool(k) as pool:
            res = pool.map(_one, [(s, args.steps) for s in range(k)])
        wall = time.perf_counter() - t0
        units = sum(r[0] for r in res)
        slowest = max(r[1] for r in res)
        rows.append({"processes": k, "cores": k, "value": units / slowest,
                     "unit": "agent-env-steps/s",
                     "per_process_s": [round(r[1], 3) for r in res], "wall_s": round(wall, 2),
                     "sample": "%d agent-env-steps per process (1 env x %d steps x 5 agents)"
                               % (res[0][0], args.steps)})
        print(rows[-1])
    out = {"what": "reference gridworld C4 Python loop (CoordinatedMultiBuildingControlEnv "
                   "restated as oracle/make_golden.CoordinatedEnv), stub PF, stdout to devnull",
           "host": "build container (%s, %d CPUs), not the GPU host" % (platform.processor() or
                                                                       platform.machine(),
                                                                       os.cpu_count()),
           "rows": rows}
    path = os.path.join(REPO, "profiles", "ref_cpu_loop.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
