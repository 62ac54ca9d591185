"""C4 at 65,536 envs: exact fixed point vs OpenDSS rule (fast kernels, with
the response table or -- opendss_notable -- every env solved) vs OpenDSS rule
(general kernel) -- us/step over a driver-shaped region and the PF kernel's
event-timed mean.  Usage: python tools/gpu/od_probe.py [--steps 200]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from powergridworld_amd import _lib  # noqa: E402
from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config  # noqa

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--n", type=int, default=65536)
ap.add_argument("--modes", default="exact,opendss,opendss_notable,opendss_general")
ap.add_argument("--max-iter", type=int, default=0, help="opendss only: cap the iterations (results "
                                                          "change), for the per-iteration cost")
ap.add_argument("--nobound", action="store_true", help="opendss only: zero bound constants (timing only)")
ap.add_argument("--hist", type=int, default=0, help="after timing: per-step max iterations over HIST steps")
ap.add_argument("--rows", default="", help="opendss only: 'none' (no check row evaluated; results wrong) "
                                         "or 'all' (every row every iteration), for phase costs")
ap.add_argument("--sparse", type=int, default=None, help="opendss only: pgw_pf_od.sparse_envs (0 default, "
                                                         "-1 never, 64 always)")
a = ap.parse_args()
dev = torch.device("cuda:0")
n = a.n
gen = torch.Generator(dev).manual_seed(0)
pool = torch.empty((16, 5, 8, n), dtype=torch.float64, device=dev).uniform_(-1, 1, generator=gen).transpose(2, 3)
for mode in a.modes.split(","):
    conv = "exact" if mode == "exact" else "opendss"
    env = CoordinatedMultiBuildingControlEnv(**make_c4_config(pf_convergence=conv, pf_general=mode.endswith("general")),
                                             num_envs=n, device=dev, fused=True)
    if mode == "opendss_notable":
        env.pf_solver.od_table = False
    if a.rows and mode == "opendss":
        od = env.pf_solver._od_proto
        od.n_rep = 0 if a.rows == "none" else od.n_rows
        if a.rows == "none":
            od.n_rows = 0
        env.pf_solver._tables_cache.clear()
        env._fused["step_cache"].clear()
    if a.sparse is not None and mode == "opendss":
        env.pf_solver._od_proto.sparse_envs = a.sparse
        env.pf_solver._tables_cache.clear()
        env._fused["step_cache"].clear()
    if a.nobound and mode == "opendss":      # bounds that always decide (timing only)
        od = env.pf_solver._od_proto
        od.gmax = od.gamma = od.gsrc = od.eps = 0.0
        env.pf_solver._tables_cache.clear()
        env._fused["step_cache"].clear()
    if a.max_iter and mode == "opendss":
        s = env.pf_solver
        s.params.max_iter = s.max_iter = a.max_iter
        s._step_cache.clear()
        s._tables_cache.clear()
        s.tables_version += 1
        env._fused["step_cache"].clear()
    env.reset()
    k = [0]

    def run(m):
        for _ in range(m):
            _, _, d, _ = env.step(pool[k[0] % 16])
            k[0] += 1
            if d["__all__"]:
                env.reset()
    run(30)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(a.steps)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / a.steps * 1e6
    _lib.check(_lib.lib().pgw_timing_start(1))
    run(64)
    torch.cuda.synchronize()
    tot = (_lib.C.c_double * 6)()
    cnt = (_lib.C.c_int64 * 6)()
    _lib.check(_lib.lib().pgw_timing_stop(tot, cnt))
    ks = {nm: round(tot[i] / cnt[i] * 1e3, 2) for i, nm in enumerate(("agents", "coord_pf", "pf_solve", "-", "ma", "pf_general")) if cnt[i]}
    it = env.pf_solver.iterations.abs()
    if a.hist:            # per-step max / mean iterations over a pass (one sync per step)
        hist, seq, seq2 = {}, [], []
        for _ in range(a.hist):
            run(1)
            its = env.pf_solver.iterations.abs()
            mx, mn = int(its.max()), int(its.min())
            hist[mx] = hist.get(mx, 0) + 1
            seq.append("%d%d" % (mn, mx))
            early = (its < mx).view(-1, 64).sum(1)           # per wave: envs stopping before the step's max
            seq2.append("%d/%d" % (int((early > 0).sum()), int(early.max())))
        print("  per-step max iterations over %d steps: %s" % (a.hist, dict(sorted(hist.items()))))
        print("  per-step (min, max) iterations in order: " + " ".join(seq))
        print("  per-step waves with an env stopping before the max / most such envs in one wave: " +
              " ".join(seq2))
    tag = mode + ("/" + a.rows if a.rows and mode == "opendss" else "") + \
        ("/max%d" % a.max_iter if a.max_iter and mode == "opendss" else "") + \
        ("/nobound" if a.nobound and mode == "opendss" else "")
    print("%-16s %7.2f us/step  kernels %s  iters mean %.3f max %d  kernel=%s" %
          (tag, us, ks, it.double().mean().item(), it.max().item(), env._fused["kernel"]), flush=True)
    if getattr(env.pf_solver, "od_resp_stats", None):
        print("  response tables: %s" % env.pf_solver.od_resp_stats, flush=True)
    del env
    torch.cuda.synchronize()
