"""Wall time of env.reset() (host + the GPU work it queues) for C3, C4 and HET,
synchronised, after warm episodes: resets fall inside the benches' timed loops."""
import os
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tools"))
import bench_configs as bc  # noqa: E402
from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config  # noqa: E402
from powergridworld_amd.multiagent_env import MultiAgentEnv  # noqa: E402
from powergridworld_amd.scenarios.heterogeneous import make_env_config  # noqa: E402
from powergridworld_amd import MultiComponentEnv  # noqa: E402
from powergridworld_amd.agents import EnergyStorageEnv, EVChargingEnv, FiveZoneROMThermalEnergyEnv, PVEnv  # noqa: E402

dev = torch.device("cuda", 0)


def timeit(label, fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    print("%-28s reset: min %8.1f us, median %8.1f us" % (label, min(ts), sorted(ts)[len(ts) // 2]))


comps = [
    {"name": "building", "cls": FiveZoneROMThermalEnergyEnv, "config": {}},
    {"name": "pv", "cls": PVEnv, "config": {"profile_csv": "pv_profile.csv", "scaling_factor": 40.}},
    {"name": "storage", "cls": EnergyStorageEnv, "config": {}},
    {"name": "ev", "cls": EVChargingEnv,
     "config": dict(num_vehicles=100, minutes_per_step=5, max_charge_rate_kw=7.,
                    peak_threshold=250., vehicle_multiplier=5., rescale_spaces=True)},
]
c3 = MultiComponentEnv(name="mc", components=comps, num_envs=16384, device=dev)
init = torch.empty(16384, dtype=torch.float64, device=dev).uniform_(3.0, 50.0)
timeit("C3 (16384)", lambda: c3.reset(init_storage=init))
c4 = CoordinatedMultiBuildingControlEnv(**make_c4_config(), num_envs=65536, device=dev, fused=True)
timeit("C4 fused (65536)", lambda: c4.reset())
het = MultiAgentEnv(**make_env_config(), num_envs=65536, device=dev)
timeit("HET (65536)", lambda: het.reset())
import cProfile, pstats  # noqa: E402,E401
for label, env, fn in (("C4", c4, lambda: c4.reset()), ("C3", c3, lambda: c3.reset(init_storage=init))):
    # host time of reset alone with a deep GPU queue in front of it: a reset
    # that synchronises waits for the queue
    x = torch.zeros(1 << 24, dtype=torch.float64, device=dev)
    for _ in range(200):
        x.mul_(1.0000001)
    t0 = time.perf_counter()
    fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("%s reset host %.1f us (queue drain after: %.1f us)" % (label, (t1 - t0) * 1e6, (t2 - t1) * 1e6))
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    c4.reset()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
