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


_BARRIER = None


def _init(barrier):
    global _BARRIER
    _BARRIER = barrier


def _one(args):
    seed, steps, reps = args
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

    def episode():
        env.reset()
        t0 = time.perf_counter()
        for t in range(steps):
            _, _, d, _ = env.step({nm: {"building": acts[t, a, :6], "pv": acts[t, a, 6:7],
                                        "storage": acts[t, a, 7:8]} for a, nm in enumerate(names)})
            if d["__all__"]:
                env.reset()
        return time.perf_counter() - t0
    with contextlib.redirect_stdout(sink):
        episode()                                   # warm-up episode (imports, first-call costs)
        if _BARRIER is not None:
            _BARRIER.wait()                         # every process times at the same time
        times = [episode() for _ in range(reps)]
    return len(names) * steps, times


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=286)
    ap.add_argument("--reps", type=int, default=3, help="timed episodes per process (after one warm-up)")
    ap.add_argument("--procs", type=int, nargs="+", default=[1, 8])
    args = ap.parse_args()
    import multiprocessing as mp
    import statistics
    ctx = mp.get_context("fork")
    rows = []
    for k in args.procs:
        t0 = time.perf_counter()
        barrier = ctx.Barrier(k)
        with ctx.Pool(k, initializer=_init, initargs=(barrier,)) as pool:
            res = pool.map(_one, [(s, args.steps, args.reps) for s in range(k)])
        wall = time.perf_counter() - t0
        units = sum(r[0] for r in res)
        med = [statistics.median(r[1]) for r in res]
        rows.append({"processes": k, "cores": k, "value": units / max(med),
                     "unit": "agent-env-steps/s",
                     "per_process_median_s": [round(x, 3) for x in med],
                     "per_process_episodes_s": [[round(x, 3) for x in r[1]] for r in res],
                     "wall_s": round(wall, 2),
                     "sample": "%d agent-env-steps per episode per process (1 env x %d steps x 5 agents); "
                               "one warm-up episode, then %d timed episodes started together (barrier); "
                               "value = all processes' units / the slowest process's median episode"
                               % (res[0][0], args.steps, args.reps)})
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
