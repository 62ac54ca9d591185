"""Per-wave phase trace of the MC step (C3, k_mc_step) and the fused
multi-agent step (HET, k_ma_step): which wave of a block is its critical path
-- the building wave, the EV walk (one lane or its split groups), PV / storage
-- step by step over an episode.  pgw_debug_mc_trace switches the launches to
their trace instantiations (lane 0 of each wave stamps wall_clock64(), 100 MHz,
at its phase boundaries, pgw_components.hip mc_trace).

Usage: python tools/gpu/mc_trace.py [--configs C3,HET] [--every 12]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from powergridworld_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="C3,HET")
ap.add_argument("--every", type=int, default=12)
a = ap.parse_args()
dev = torch.device("cuda:0")


def summarize(tag, buf, n_waves, roles, extra=""):
    t = buf.view(-1, 16, 8)[:, :n_waves].cpu().numpy().astype(np.float64) / 100.0   # us
    t0 = t[:, :, 0].min()
    start = t[:, :, 0].min(1) - t0                     # block start
    raw6 = buf.view(-1, 16, 8)[:, :n_waves, 6].cpu().numpy()
    end = np.where(raw6 != 0, t[:, :, 6], -np.inf).max(1) - t0   # the sums written (by whichever wave)
    comp = t[:, :, 2] - t[:, :, 0]                     # each wave's own work
    wait = t[:, :, 5] - t[:, :, 2]                     # each wave's wait at the barriers
    line = "%s %s span %.2f  block start p50 %.2f max %.2f  block life p50 %.2f max %.2f |" % (
        tag, extra, end.max(), np.median(start), start.max(), np.median(end - start), (end - start).max())
    for w in range(n_waves):
        line += " %s %.2f/%.2f" % (roles[w], np.median(comp[:, w]), comp[:, w].max())
    raw = buf.view(-1, 16, 8)[:, :n_waves].cpu().numpy()
    if (raw[:, :, 4] != 0).any():                     # the EV finisher: fold + finish after its own walk
        fin = raw[:, :, 4] != 0
        fold = (np.where(fin, t[:, :, 4], 0).max(1) - np.where(fin, t[:, :, 2], 0).max(1))
        line += " | fold+finish %.2f" % np.median(fold)
    for w in range(n_waves):                          # EV group waves: the first pair's chunks
        if roles[w].startswith("ev") and (raw[:, w, 3] != 0).all() and (raw[:, w, 7] != 0).all():
            line += " | %s to A %.2f B %.2f" % (roles[w], np.median(t[:, w, 3] - t[:, w, 0]),
                                               np.median(t[:, w, 7] - t[:, w, 3]))
    bw = [w for w in range(n_waves) if (raw[:, w, 3] != 0).all() and roles[w].startswith("bld")]
    if bw:                                            # the building wave's phases
        w = bw[0]
        line += " | bld loads %.2f state+reward %.2f obs %.2f" % (
            np.median(t[:, w, 3] - t[:, w, 0]), np.median(t[:, w, 7] - t[:, w, 3]), np.median(t[:, w, 2] - t[:, w, 7]))
    crit = np.bincount(np.argmax(t[:, :, 2], 1), minlength=n_waves)
    line += " | last-to-finish wave counts %s" % crit.tolist()
    print(line, flush=True)
    return end.max()


def c3(every):
    from bench_configs import c3_env
    n = 16384
    env, acts = c3_env(dev, n)
    env.reset()
    buf = torch.zeros((n // 64) * 128, dtype=torch.int64, device=dev)
    spans = []
    _lib.check(_lib.lib().pgw_debug_mc_trace(_lib.dptr(buf)))
    try:
        for k in range(286):
            buf.zero_()
            env.step(acts[k % len(acts)])
            torch.cuda.synchronize()
            t = buf.view(-1, 16, 8).cpu().numpy()
            nw = int((t[0, :, 0] != 0).sum())
            if k % every == 0:
                roles = (["bld", "pv", "sto", "ev0"] + ["ev%d" % g for g in range(1, 8)])[:nw]
                spans.append(summarize("C3 step %3d" % k, buf, nw, roles, "waves %d" % nw))
    finally:
        _lib.check(_lib.lib().pgw_debug_mc_trace(None))
    print("C3 sampled spans: mean %.2f us" % np.mean(spans), flush=True)


def het(every):
    from powergridworld_amd.multiagent_env import MultiAgentEnv
    from powergridworld_amd.scenarios.heterogeneous import make_env_config
    n = 65536
    env = MultiAgentEnv(**make_env_config(), num_envs=n, device=dev)
    gen = torch.Generator(dev).manual_seed(0)
    acts = []
    for _ in range(8):
        acts.append({ag.name: ({c.name: torch.empty((n, c.action_space.shape[0]), dtype=torch.float64,
                                                     device=dev).uniform_(-1, 1, generator=gen)
                                for c in ag.envs} if hasattr(ag, "envs") else
                               torch.empty((n, ag.action_space.shape[0]), dtype=torch.float64,
                                           device=dev).uniform_(-1, 1, generator=gen))
                     for ag in env.agents})
    env.reset()
    args = env._ma["args"]
    kind_name = {0: "bld", 1: "pv", 2: "sto", 3: "ev"}
    roles = ["+".join(kind_name[args.comp[args.wave_slot[args.wave_first[w] + i]].kind]
                      for i in range(args.wave_count[w])) for w in range(args.n_waves)]
    buf = torch.zeros((n // 64) * 128, dtype=torch.int64, device=dev)
    spans = []
    _lib.check(_lib.lib().pgw_debug_mc_trace(_lib.dptr(buf)))
    try:
        for k in range(286):
            buf.zero_()
            env.step(acts[k % len(acts)])
            torch.cuda.synchronize()
            t = buf.view(-1, 16, 8).cpu().numpy()
            nw = int((t[0, :, 0] != 0).sum())
            if k % every == 0:
                spans.append(summarize("HET step %3d" % k, buf, nw, roles, "waves %d" % nw))
    finally:
        _lib.check(_lib.lib().pgw_debug_mc_trace(None))
    print("HET sampled spans: mean %.2f us" % np.mean(spans), flush=True)


for c in a.configs.split(","):
    {"C3": c3, "HET": het}[c](a.every)
