"""Probe: k_ma_step duration for subsets of the heterogeneous scenario's agents
(library events, every launch) -- which component bounds the fused step."""
import ctypes
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
from powergridworld_amd import _lib  # noqa: E402
from powergridworld_amd.multiagent_env import MultiAgentEnv  # noqa: E402
from powergridworld_amd.scenarios.heterogeneous import make_env_config  # noqa: E402

N = 65536
MultiAgentEnv._fusable = lambda self: "probe: the multi-agent step only"
dev = torch.device("cuda", 0)
lib = _lib.lib()


def run(names, steps=100, fused=True):
    cfg = make_env_config()
    cfg["agents"] = [a for a in cfg["agents"] if a["name"] in names]
    env = MultiAgentEnv(**cfg, num_envs=N, device=dev, fused=fused)
    assert (env._ma is not None) == fused
    gen = torch.Generator(dev).manual_seed(0)
    acts = []
    for _ in range(8):
        acts.append({a.name: ({c.name: torch.empty((N, c.action_space.shape[0]), dtype=torch.float64,
                                                    device=dev).uniform_(-1, 1, generator=gen) for c in a.envs}
                              if hasattr(a, "envs") else
                              torch.empty((N, a.action_space.shape[0]), dtype=torch.float64,
                                          device=dev).uniform_(-1, 1, generator=gen)) for a in env.agents})
    env.reset()
    for k in range(20):
        env.step(acts[k % 8])
    torch.cuda.synchronize()
    _lib.check(lib.pgw_timing_start(1))
    for k in range(steps):
        _, _, d, _ = env.step(acts[k % 8])
        if d["__all__"]:
            env.reset()
    torch.cuda.synchronize()
    tot, cnt = (ctypes.c_double * 8)(), (ctypes.c_int64 * 8)()
    _lib.check(lib.pgw_timing_stop(tot, cnt))
    print("%-40s waves=%d  k_ma_step %.2f us  k_pf_solve %.2f us" % (
        "+".join(names) + ("" if fused else " (generic)"), env._ma["args"].n_waves if fused else 0, tot[4] / max(cnt[4], 1) * 1e3, tot[2] / max(cnt[2], 1) * 1e3),
        flush=True)


for names in (["building"], ["pv"], ["ev-charging"], ["building", "pv"], ["pv", "ev-charging"],
              ["building", "ev-charging"], ["building", "pv", "ev-charging"]):
    run(names)
run(["building", "pv", "ev-charging"], fused=False)
