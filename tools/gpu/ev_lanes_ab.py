"""A/B of the EV step: the one-lane walk (pgw_ev_step, [V, N] requirements)
against lanes over vehicles (pgw_ev_step_lanes, env-major [N, row]) on the same
pre-step state, step info and actions, over an episode.  Prints the largest
differences per output and, per config, the two kernels' mean times (HIP
events around each launch, the launches back to back on one stream).
Usage: python tools/gpu/ev_lanes_ab.py [steps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from powergridworld_amd import _lib  # noqa
from powergridworld_amd.agents import EVChargingEnv  # noqa
from powergridworld_amd.base import as_action  # noqa

dev = torch.device("cuda", 0)
STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 287
lib = _lib.lib()
lib.pgw_ev_row.restype = _lib.C.c_int32


def to_rows(x, row):            # [V, N] -> [N, row]
    V, n = x.shape
    out = torch.zeros((n, row), dtype=x.dtype, device=x.device)
    out[:, :V] = x.t()
    return out


def run(V, n, randomize=False, seed=0):
    env = EVChargingEnv(num_vehicles=V, minutes_per_step=5, max_charge_rate_kw=7., peak_threshold=250.,
                        vehicle_multiplier=5., rescale_spaces=True, randomize=randomize, num_envs=n, device=dev)
    if randomize:
        env.seed(seed)
    env.reset()
    row = int(lib.pgw_ev_row(V))
    gen = torch.Generator(dev).manual_seed(seed)
    st = _lib.stream_ptr(dev)
    worst = {}
    t_old, t_new, cnt = 0.0, 0.0, 0
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    est = est_ = None
    if randomize:
        est, est_ = to_rows(env._env_start, row), to_rows(env._env_endp, row)
    for k in range(STEPS):
        if env.is_terminal():
            break
        a = torch.rand((n, 1), dtype=torch.float64, device=dev, generator=gen) * 2.2 - 1.1
        s = env._step_info_at(env.time_index, env._prev_window)[0]
        if randomize:
            s.env_start, s.env_endp = est.data_ptr(), est_.data_ptr()
        req0, chg0 = env.req.clone(), env.charging.clone()
        obs0, rp0, rew0 = env._new_obs(6), torch.zeros(n, dtype=torch.float64, device=dev), \
            torch.zeros(n, dtype=torch.float64, device=dev)
        req1, chg1 = to_rows(env.req, row), env.charging.clone()
        obs1, rp1, rew1 = env._new_obs(6), torch.zeros(n, dtype=torch.float64, device=dev), \
            torch.zeros(n, dtype=torch.float64, device=dev)
        am = env._mat(as_action(a, n, 1, dev, torch.float64))
        s0 = s
        if randomize:
            s0 = type(s).from_buffer_copy(s)
            s0.env_start, s0.env_endp = env._env_start.data_ptr(), env._env_endp.data_ptr()
        torch.cuda.synchronize()
        ev[0].record()
        _lib.check(lib.pgw_ev_step(env.params, s0, n, am, _lib.dptr(env._endp_dev), req0.data_ptr(),
                                   chg0.data_ptr(), env._mat(obs0), rp0.data_ptr(), rew0.data_ptr(), st))
        ev[1].record()
        _lib.check(lib.pgw_ev_step_lanes(env.params, s, n, am, _lib.dptr(env._endp_dev), req1.data_ptr(),
                                         chg1.data_ptr(), env._mat(obs1), rp1.data_ptr(), rew1.data_ptr(), st))
        ev[2].record()
        torch.cuda.synchronize()
        env.step(a)
        if k >= 3:
            t_old += ev[0].elapsed_time(ev[1])
            t_new += ev[1].elapsed_time(ev[2])
            cnt += 1
        rel = lambda x, y: ((x - y).abs() / (1e-300 + y.abs().clamp_min(1e-12))).max().item()
        d = {"obs": rel(obs1, obs0), "rp": rel(rp1, rp0), "rew": rel(rew1, rew0),
             "req": (req1[:, :V] - req0.t()).abs().max().item(),
             "chg": int((chg1 != chg0).sum()),
             "nact": (obs1[:, 1] - obs0[:, 1]).abs().max().item(),
             "env": rel(obs0, env._obs)}
        for key, v in d.items():
            worst[key] = max(worst.get(key, 0), v)
    print("V=%d n=%d randomize=%s row=%d steps=%d: worst %s | us per launch: walk %.2f  lanes %.2f" % (
        V, n, randomize, row, k + 1, {k_: ("%.3g" % v) for k_, v in worst.items()}, 1e3 * t_old / max(cnt, 1),
        1e3 * t_new / max(cnt, 1)), flush=True)
    return worst


if __name__ == "__main__":
    for V, n, rnd in ((100, 16384, False), (25, 65536, False), (10, 65536, False), (100, 65536, False),
                      (40, 8192, True), (200, 4096, False)):
        run(V, n, rnd)
