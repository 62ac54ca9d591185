"""Host cost of the C3 step (MultiComponentEnv building + PV + storage + EV(100))
at a tiny batch (GPU far ahead) and at 16384: the whole env.step, the bare
pgw_mc_agent_step call with the cached arguments, and a cProfile of the loop."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from powergridworld_amd import MultiComponentEnv, _lib
from powergridworld_amd.agents import EnergyStorageEnv, EVChargingEnv, FiveZoneROMThermalEnergyEnv, PVEnv

comps = [
    {"name": "building", "cls": FiveZoneROMThermalEnergyEnv, "config": {}},
    {"name": "pv", "cls": PVEnv, "config": {"profile_csv": "pv_profile.csv", "scaling_factor": 40.}},
    {"name": "storage", "cls": EnergyStorageEnv, "config": {}},
    {"name": "ev", "cls": EVChargingEnv,
     "config": dict(num_vehicles=100, minutes_per_step=5, max_charge_rate_kw=7.,
                    peak_threshold=250., vehicle_multiplier=5., rescale_spaces=True)},
]
dev = torch.device("cuda", 0)
for n in (256, 16384):
    env = MultiComponentEnv(name="mc", components=comps, num_envs=n, device=dev)
    dims = {"building": 6, "pv": 1, "storage": 1, "ev": 1}
    act = {c: torch.zeros((n, d), dtype=torch.float64, device=dev) for c, d in dims.items()}
    env.reset()

    def run(k):
        for _ in range(k):
            _, _, d, _ = env.step(act)
            if d:
                env.reset()

    run(300)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(572)
    torch.cuda.synchronize()
    print("n=%d env.step: %.1f us/step" % (n, (time.perf_counter() - t0) / 572 * 1e6))
lib, st = _lib.lib(), _lib.stream_ptr(dev)
args = env._mc_args
for rep in range(2):
    t0 = time.perf_counter()
    for _ in range(2000):
        lib.pgw_mc_agent_step(args, env.num_envs, st)
    torch.cuda.synchronize()
    print("bare pgw_mc_agent_step at n=%d: %.1f us/call" % (env.num_envs, (time.perf_counter() - t0) / 2000 * 1e6))
pr = cProfile.Profile()
pr.enable()
run(572)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
