"""Throughput of the BASELINE configs other than the headline C4 (BASELINE.md
section 4): C2 = EnergyStorageEnv defaults at batch 4096, C3 = the
MultiComponentEnv building + PV + storage + EV(100 vehicles) at batch 16384,
and HET = the reference's 3-agent heterogeneous scenario (scenarios/
heterogeneous.py) and HS = the Home-Steward house (base_hs.py) at 65536.  Each step goes through the public API
with actions resident in HBM (a pool of pre-generated batches); episodes reset
inside the timed region.  One JSON line per config.

Usage: python tools/bench_configs.py [--configs C2,C3,HET,HETG,HS,...] [--steps K] [--warmup W]
(HET: OpenDSS's snap-solve rule, the default, with its response table; HETS:
every env solved; HETX: the exact fixed point; HETG: the heterogeneous scenario
on the generic path, fused=False; C3F / C3G8F:
C3 with fp32 storage (pgw_mc_agent_step_f32); C3L: C3 at
65 536 envs; C2Gk / C3Gk: the step replayed from captured hipGraphs of k steps,
C3 through the device clocks; C3Pk / HSPk: captured once per episode position,
powergridworld_amd/graph.py)
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# algorithmic HBM bytes per agent-env-step
BYTES = {"C2": 48, "C3": 1990}


def timed_loop(env, step, reset, steps, warmup):
    reset()
    for _ in range(warmup):
        if step():
            reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        if step():
            reset()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def graph_steps(env, acts, per, reset, clocked=False):
    """Captured steps (powergridworld_amd/graph.py) over the action pool: one
    graph per pool entry (per = 1: as if the policy wrote into one of the pool's
    buffers), or graphs of `per` consecutive pool entries (open-loop rollout).
    Returns step() -> done, advancing `per` env steps per call."""
    pool = len(acts)
    kw = {"clocked": True} if clocked else {}
    graphs = [env.capture_step(acts[i] if per == 1 else [acts[(i + j) % pool] for j in range(per)], steps=per, **kw)
              for i in range(0, pool, per)]
    reset()
    k = [0]

    def step():
        done = graphs[k[0] % len(graphs)]()[2]
        k[0] += 1
        return done
    return step


def bench_c2(dev, steps, warmup, n=4096, pool=64, graph=0):
    from powergridworld_amd.agents import EnergyStorageEnv
    env = EnergyStorageEnv(num_envs=n, device=dev)
    gen = torch.Generator(dev).manual_seed(0)
    acts = torch.empty((pool, n, 1), dtype=torch.float64, device=dev).uniform_(-1, 1, generator=gen)
    init = torch.empty(n, dtype=torch.float64, device=dev).uniform_(3.0, 50.0, generator=gen)
    k = [0]

    def step():
        _, _, done, _ = env.step(acts[k[0] % pool])
        k[0] += 1
        return done

    reset = lambda: env.reset(init_storage=init)
    if graph:
        step = graph_steps(env, list(acts), graph, reset)
        steps, warmup = steps // graph, warmup // graph
    dt = timed_loop(env, step, reset, steps, warmup)
    steps *= max(graph, 1)
    return dict(config="C2" + ("G%d" % graph if graph else ""),
                workload="EnergyStorageEnv defaults" + (", %d-step captured graphs" % graph if graph else ""),
                batch=n, agents=1, steps=steps, seconds=dt)


def c3_env(dev, n, pool=16, dtype=torch.float64):
    """The C3 agent and a pool of pre-generated action dicts (HBM resident)."""
    from powergridworld_amd import MultiComponentEnv
    from powergridworld_amd.agents import EnergyStorageEnv, EVChargingEnv, FiveZoneROMThermalEnergyEnv, PVEnv
    comps = [
        {"name": "building", "cls": FiveZoneROMThermalEnergyEnv, "config": {}},
        {"name": "pv", "cls": PVEnv, "config": {"profile_csv": "pv_profile.csv", "scaling_factor": 40.}},
        {"name": "storage", "cls": EnergyStorageEnv, "config": {}},
        {"name": "ev", "cls": EVChargingEnv,
         "config": dict(num_vehicles=100, minutes_per_step=5, max_charge_rate_kw=7.,
                        peak_threshold=250., vehicle_multiplier=5., rescale_spaces=True)},
    ]
    env = MultiComponentEnv(name="mc", components=comps, num_envs=n, device=dev, dtype=dtype)
    gen = torch.Generator(dev).manual_seed(0)
    dims = {"building": 6, "pv": 1, "storage": 1, "ev": 1}
    acts = [{c: torch.empty((n, d), dtype=dtype, device=dev).uniform_(-1, 1, generator=gen)
             for c, d in dims.items()} for _ in range(pool)]
    return env, acts


def bench_c3(dev, steps, warmup, n=16384, pool=16, graph=0, clocked=True, dtype=torch.float64):
    env, acts = c3_env(dev, n, pool, dtype)
    gen = torch.Generator(dev).manual_seed(1)
    init = torch.empty(n, dtype=dtype, device=dev).uniform_(3.0, 50.0, generator=gen)
    k = [0]

    def step():
        _, _, done, _ = env.step(acts[k[0] % pool])
        k[0] += 1
        return done

    reset = lambda: env.reset(init_storage=init)
    if graph:
        # (the episode's 287 steps are not a multiple of `graph`: before a call
        # that would pass the end, the env resets, as done would make it)
        reset()
        gstep = graph_steps(env, acts, graph, reset, clocked)

        def step():
            if env._ep_step + graph > 287:
                reset()
            return gstep()
        steps, warmup = steps // graph, warmup // graph
        if not clocked:
            # every (graph, position) pair is captured on first use: warm up
            # until the pool's graphs have met every position (the pool cycles
            # with period len(graphs) calls, an episode is 287 // graph calls)
            warmup = max(warmup, (pool // graph) * (287 // graph + 1))
    dt = timed_loop(env, step, reset, steps, warmup)
    steps *= max(graph, 1)
    return dict(config="C3" + ("L" if n != 16384 else "") + (("G%d" if clocked else "P%d") % graph if graph else "")
                + ("F" if dtype == torch.float32 else ""),
                workload="MC building+PV+storage+EV(100 vehicles)" + (
                    ", %d-step captured graphs%s" % (graph, "" if clocked else " per episode position")
                    if graph else ""),
                batch=n, agents=1, steps=steps, seconds=dt)


def bench_het(dev, steps, warmup, n=65536, pool=16, fused="auto", conv="opendss", table=True, vrec=True, qrec=True,
              rrows=True):
    from powergridworld_amd.scenarios.heterogeneous import make_env_config
    from powergridworld_amd.multiagent_env import MultiAgentEnv
    env = MultiAgentEnv(**make_env_config(pf_convergence=conv), num_envs=n, device=dev, fused=fused)
    env.pf_solver.od_table = table
    if hasattr(env.pf_solver, "od_node_records"):
        env.pf_solver.od_node_records = vrec
        env.pf_solver.od_row_records = qrec
        env.pf_solver.od_record_rows = rrows
        env.pf_solver._tables_cache.clear()
        env.pf_solver._od_qinfo.clear()
    gen = torch.Generator(dev).manual_seed(0)
    acts = []
    for _ in range(pool):
        acts.append({a.name: ({c.name: torch.empty((n, c.action_space.shape[0]), dtype=torch.float64,
                                                    device=dev).uniform_(-1, 1, generator=gen)
                               for c in a.envs} if hasattr(a, "envs") else
                              torch.empty((n, a.action_space.shape[0]), dtype=torch.float64,
                                          device=dev).uniform_(-1, 1, generator=gen))
                     for a in env.agents})
    k = [0]

    def step():
        _, _, dones, _ = env.step(acts[k[0] % pool])
        k[0] += 1
        return dones["__all__"]

    dt = timed_loop(env, step, env.reset, steps, warmup)
    return dict(config=("HET" if fused else "HETG") + ("X" if conv == "exact" else "") + ("" if table else "S")
                + ("" if vrec else "V") + ("" if qrec else "Q") + ("" if rrows else "R"),
                workload="3-agent heterogeneous (MC building, grid-aware PV farm, EV 25x40) + IEEE-13 PF, "
                         + ("fused multi-agent step (pgw_ma_step)" if env._ma is not None else "generic path"),
                pf_convergence=conv, pf_response_table=bool(table and conv == "opendss"),
                batch=n, agents=3, steps=steps, seconds=dt)


def bench_hs(dev, steps, warmup, n=65536, pool=16, graph=0):
    from powergridworld_amd.base_hs import HSMultiComponentEnv
    from powergridworld_amd.scenarios.heterogeneous_hs import make_env_config
    env = HSMultiComponentEnv(**make_env_config(), num_envs=n, device=dev)
    gen = torch.Generator(dev).manual_seed(0)
    acts = torch.empty((pool, n, len(env.envs)), dtype=torch.float64, device=dev).uniform_(-1, 1, generator=gen)
    k = [0]

    def step():
        _, _, done, _ = env.step(acts[k[0] % pool])
        k[0] += 1
        return done

    if graph:
        # per-position graphs of `graph` steps over the pool (as C3's); before
        # a call that would pass the data's end the house resets
        env.reset()
        gstep = graph_steps(env, list(acts), graph, env.reset)
        L = env._hs_steps()

        def step():
            if env._hs_step_k() + graph > L:
                env.reset()
            return gstep()
        steps, warmup = steps // graph, max(warmup // graph, (pool // graph) * (L // graph + 1))
    dt = timed_loop(env, step, env.reset, steps, warmup)
    steps *= max(graph, 1)
    return dict(config="HS" + ("P%d" % graph if graph else ""),
                workload="Home-Steward house (PV, battery, EV, devices; shipped JSON scenario)" + (
                    ", %d-step captured graphs per episode position" % graph if graph else ""),
                batch=n, agents=1, steps=steps, seconds=dt)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C3,HET,HS")
    ap.add_argument("--steps", type=int, default=572)
    ap.add_argument("--warmup", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    fns = {"C2": bench_c2, "C3": bench_c3, "HET": bench_het, "HS": bench_hs,
           "HETG": lambda *a: bench_het(*a, fused=False),
           "HETX": lambda *a: bench_het(*a, conv="exact"),
           "HETS": lambda *a: bench_het(*a, table=False),
           "HETV": lambda *a: bench_het(*a, vrec=False),
           "HETQ": lambda *a: bench_het(*a, qrec=False),
           "HETR": lambda *a: bench_het(*a, rrows=False),
           "C2G1": lambda *a: bench_c2(*a, graph=1), "C2G8": lambda *a: bench_c2(*a, graph=8),
           "C3G1": lambda *a: bench_c3(*a, graph=1), "C3G8": lambda *a: bench_c3(*a, graph=8),
           "C3P1": lambda *a: bench_c3(*a, graph=1, clocked=False),
           "C3P8": lambda *a: bench_c3(*a, graph=8, clocked=False),
           "C3L": lambda *a: bench_c3(*a, n=65536),
           "C3F": lambda *a: bench_c3(*a, dtype=torch.float32),
           "C3G8F": lambda *a: bench_c3(*a, graph=8, dtype=torch.float32),
           "HSP8": lambda *a: bench_hs(*a, graph=8)}
    for name in args.configs.split(","):
        r = fns[name](dev, args.steps, args.warmup)
        units = r["batch"] * r["agents"] * r["steps"]
        r["value"] = units / r["seconds"]
        r["unit"] = "agent-env-steps/s"
        r["us_per_step"] = r["seconds"] / r["steps"] * 1e6
        if name[:2] in BYTES:
            r["step_level_hbm_gbs"] = BYTES[name[:2]] * units / r["seconds"] / 1e9
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
