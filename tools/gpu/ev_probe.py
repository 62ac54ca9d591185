"""Probe: EV-only fused multi-agent step (k_ma_step) vs the number of vehicles,
library events -- how much of the EV wave is per-vehicle work."""
import copy
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from powergridworld_amd import _lib  # noqa: E402
from powergridworld_amd.multiagent_env import MultiAgentEnv  # noqa: E402
from powergridworld_amd.scenarios.heterogeneous import make_env_config  # noqa: E402

N = 65536
dev = torch.device("cuda", 0)
lib = _lib.lib()
for nv, mult in ((1, 40.), (8, 40.), (25, 40.), (64, 10.), (100, 5.)):
    cfg = make_env_config()
    ev = copy.deepcopy([a for a in cfg["agents"] if a["name"] == "ev-charging"][0])
    ev["config"]["num_vehicles"], ev["config"]["vehicle_multiplier"] = nv, mult
    cfg["agents"] = [ev]
    env = MultiAgentEnv(**cfg, num_envs=N, device=dev, fused=True)
    assert env._ma is not None
    gen = torch.Generator(dev).manual_seed(0)
    acts = [{"ev-charging": torch.empty((N, 1), dtype=torch.float64, device=dev).uniform_(-1, 1, generator=gen)}
            for _ in range(8)]
    env.reset()
    scanned = []
    for k in range(288 * 2):
        if k == 20:
            torch.cuda.synchronize()
            _lib.check(lib.pgw_timing_start(1))
        _, _, d, _ = env.step(acts[k % 8])
        st = env._ma["args"].ev_step
        scanned.append(sum(bin(st.scan[w]).count("1") for w in range(st.n_words)))
        if d["__all__"]:
            env.reset()
    torch.cuda.synchronize()
    tot, cnt = (ctypes.c_double * 8)(), (ctypes.c_int64 * 8)()
    _lib.check(lib.pgw_timing_stop(tot, cnt))
    print("vehicles %3d: mean scanned %.1f, k_ma_step %.2f us" %
          (nv, sum(scanned) / len(scanned), tot[4] / max(cnt[4], 1) * 1e3), flush=True)
