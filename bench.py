"""Benchmark: agent-env-steps/sec of the 5-agent coordinated-building scenario
with the IEEE-13 power flow (BASELINE.json config C4), batch 65,536 per GPU.

One "step" = one MultiAgentEnv.step of the whole batch through the public API
(fused path: one pgw_coord_step call.  By default, OpenDSS's snap-solve rule
as the reference runs it with the hour's certified response table, in ONE
launch: k_coord_step_od -- 5 x [building, PV, storage] per env, the power
flow's table lookup with the coordinated reward, and the snap solve of the rare
envs the table does not serve by the lookup wave (od_wave_solve);
--pf-split off: k_coord_agents_std + k_coord_pf_od (bit-identical);
--pf-convergence exact: k_coord_agents_std + k_coord_pf, the exact fixed point
with its predictor tables), actions already resident in HBM.  Episodes (286 steps) end with done["__all__"]; the following env.reset()
is inside the timed region.  Kernel durations come from HIP events the library
records around every --time-every-th launch, on the launch's stream.

Launch:  python bench.py [--gpus N --steps K --warmup W]
         N>1: under torch.distributed.run (one rank per GPU, WORLD_SIZE must
         equal N), or started directly, in which case bench.py runs
         torch.distributed.run --nproc-per-node N as a child process before
         any GPU call and exits with its return code (rank 0 prints the line).
         Weak scaling, no collective on the step path; barrier +
         max-over-ranks timing.

The CPU baseline (N=1 only) runs first, before the GPU is touched: the oracle
on 1 process and on 8 forked processes; the reference's own loop cannot run on
the GPU host, so its figures (tools/ref_cpu_loop.py, build container) are
copied in from profiles/ref_cpu_loop.json as a labelled row.
"""
import argparse
import gc
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

N_AGENTS = 5
ACT_DIM = 8
BATCH_PER_GPU = 65536
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec (6.3 measured achievable)
FP64_PEAK_TFS = 78.6         # MI355X spec, FP64 vector (= FP64 matrix); tools/micro MFMA probe 68.7
# k_coord_agents_std -- algorithmic HBM bytes per (env, agent), fp64 env-minor SoA:
#   reads  actions 8x8 + x_k 5x8 + soc 8                       = 112
#   writes x_k 5x8 + soc 8 + obs 17x8 + reward 8 + power 8     = 200
AGENT_BYTES = 112 + 200
AGENT_BYTES_F32 = AGENT_BYTES // 2       # the same items in fp32 (pgw_coord_step_f32)
# k_coord_step_od (the agents and the PF's table lookup in one launch) -- per env
# the 5 agents' bytes above plus the PF's outputs V675.3, violation (8 B each)
# and the iteration count (4 B); the agent powers stay in LDS, the node record
# (96 B) is an L2 gather, the rewards are written once (final)
STEP_OD_ENV_BYTES = 5 * AGENT_BYTES + 8 + 8 + 4
# k_coord_pf -- per env: reads 5 agent powers + 5 rewards, writes 5 rewards + v + vv + iters
PF_BYTES = 8 * (5 + 5 + 5 + 1 + 1) + 4
# k_coord_pf -- algorithmic fp64 FLOPs (m = 14 load phase elements): per fixed-point
# iteration 8 m^2 (complex matvec) + 12 m (PQ current law) + 6 m (update, |du|^2 test);
# per env once more the final currents (12 m), one node voltage (8 m + 4) and the reward.
M_ELEM = 14
PF_FLOPS_ITER = 8 * M_ELEM ** 2 + 12 * M_ELEM + 6 * M_ELEM
PF_FLOPS_ENV = 12 * M_ELEM + 8 * M_ELEM + 4 + 10
# k_coord_pf_od (OpenDSS rule, fast kernel): per compensation iteration after the
# first 8 m^2 (matvec) + 14 m (current law with the Yeq term) + 6 m (the
# square-root-free element test); once per env the exact test of the accepted
# iteration -- element magnitudes (2 x 8 per node) and the n_rep = 11 evaluated
# check rows twice (previous and new: 8 m + 4 each) -- the first iteration (14 m
# currents + 4 m affine u_1), one output row (8 m + 4) and the reward
OD_REP_ROWS = 11
OD_FLOPS_ITER = 8 * M_ELEM ** 2 + 14 * M_ELEM + 6 * M_ELEM
OD_FLOPS_ENV = 16 * M_ELEM + 2 * OD_REP_ROWS * (8 * M_ELEM + 4) + 18 * M_ELEM + 8 * M_ELEM + 4 + 10
# k_coord_pf_od with the hour's response table and its node records
# (pgw_pf_od.resp / resp_v): per env one node record (PGW_OD_VREC = 12 doubles,
# 96 B, L2-resident), the complex quadratic of V675.3 (2 x 2 FMAs), |V| and the
# reward (the response record's 720 B are read only where an env is solved)
OD_TABLE_REC_BYTES = 8 * 12
OD_TABLE_FLOPS_ENV = 8 + 4 + 10
PF_KERNEL_NAME = {"exact": "k_coord_pf<14,true,false,false>", "opendss": "k_coord_pf_od<14>"}
# (k_coord_pf_od<14>: with the hour's response table, pgw_pf_od.resp, the default)
PF_KERNEL = "k_coord_pf"              # PGW_T_COORD_PF: whichever PF kernel the step's mode runs


def pf_roofline(conv, avg_us, mean_it, n, table=False, split=False):
    """The step's PF kernel against its bound.  Exact fixed point: fp64 VALU, on
    its algorithmic flops.  OpenDSS rule with the response table: a latency
    chain (agent powers and rewards from HBM -> the env's node record from L2 ->
    the outputs and final rewards), reported as HBM GB/s of its algorithmic bytes
    with the record bytes and flops beside; without the table (od_table=False):
    fp64 VALU."""
    if conv == "opendss" and table and split:
        return {"bound": "latency", "note": "k_coord_pf_od_list: the snap solve of the envs the fused step listed "
                                            "(none when the table serves every env): a small fixed grid that reads "
                                            "the list's count and exits; its time is a dispatch's"}
    if conv == "opendss" and table:
        gbs = PF_BYTES * n / (avg_us * 1e-6) / 1e9
        return {"bound": "latency", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                "note": "latency-bound: HBM agent powers and rewards -> one %d-byte node record per env "
                        "(L2, %.1f GB/s of record gather) -> V675.3, violation, final rewards"
                        % (OD_TABLE_REC_BYTES, OD_TABLE_REC_BYTES * n / (avg_us * 1e-6) / 1e9),
                "flops_per_env": OD_TABLE_FLOPS_ENV, "l2_bytes_per_env": OD_TABLE_REC_BYTES}
    if conv == "exact":
        flops = PF_FLOPS_ITER * mean_it + PF_FLOPS_ENV
    else:
        flops = OD_FLOPS_ITER * max(mean_it - 1.0, 0.0) + OD_FLOPS_ENV
    tfs = flops * n / (avg_us * 1e-6) / 1e12
    return {"bound": "fp64 valu", "achieved": tfs, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
            "frac": tfs / FP64_PEAK_TFS, "flops_per_env": flops}


KERNELS = ("k_coord_agents_std", PF_KERNEL, "k_pf_solve", "(unused)", "k_ma_step", "k_pf_general")


def table_stats(env):
    """The hour tables' response-table statistics for the bench line."""
    st = dict(env.pf_solver.od_resp_stats)
    out = {k: st.get(k) for k in ("hours", "segments_with_breakpoints", "brackets", "unresolved_brackets",
                                  "pieces", "pieces_left_to_solve", "max_fit_err", "certified",
                                  "certified_pieces", "pieces_cut_by_certificate", "uncertified_kw",
                                  "certify_s", "build_s")}
    out["note"] = ("built on the device by the snap solve itself (pgw_pf_od_probe) about once per 24 "
                   "simulated hours, every piece certified (od_certify: Taylor-model bounds prove every band and "
                   "stopping decision constant over what its record serves; cut pieces leave a guard zone "
                   "to the solve), cached across episodes (every episode repeats the hours); build_s is the "
                   "whole build time of this run (in episode_cold), outside the timed region")
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=572)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--batch", type=int, default=BATCH_PER_GPU)
    ap.add_argument("--action-pool", type=int, default=64,
                    help="distinct pre-generated action batches cycled through (HBM resident)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-envs", type=int, default=8192)
    ap.add_argument("--cpu-sample-steps", type=int, default=143)
    ap.add_argument("--cpu-procs", type=int, default=8)
    ap.add_argument("--cpu-baseline-only", action="store_true",
                    help="(internal) print the cpu_baseline JSON and exit; bench.py runs this as a "
                         "child process so the oracle's imports stay out of the timed process")
    ap.add_argument("--time-steps", type=int, default=286,
                    help="steps of the kernel-timing pass after the timed region (every launch "
                         "HIP-event-timed; at least 8; a whole episode by default, whatever --steps)")
    ap.add_argument("--pf-convergence", choices=("opendss", "exact"), default="opendss",
                    help="the headline's power-flow stopping rule: OpenDSS's snap solve (the "
                         "reference's: loads' Yeq in Y, node-magnitude test 1e-4, 2..15 iterations) "
                         "or the exact fixed point; the other runs as variants.*_pf")
    ap.add_argument("--pf-split", choices=("on", "off"), default="on",
                    help="OpenDSS rule with node records: the one-launch step -- agents, table lookup "
                         "and the snap solve of the envs the table leaves (on) -- or the two-kernel "
                         "step (off); bit-identical")
    ap.add_argument("--no-variants", action="store_true",
                    help="skip the fp32-storage variant line (N=1 only; never the headline)")
    return ap.parse_args()


def f32_variant(conv, n, steps, warmup, pool_size, seed, dev):
    """The same C4 workload on the fp32-storage fused path (pgw_coord_step_f32:
    fp32 state/actions/outputs, fp64 arithmetic).  Reported beside
    the fp64 headline, never as it: the reference computes in fp64."""
    from powergridworld_amd import _lib
    from powergridworld_amd.scenarios.coordinated import (CoordinatedMultiBuildingControlEnv,
                                                          make_c4_config)
    env = CoordinatedMultiBuildingControlEnv(**make_c4_config(pf_convergence=conv), num_envs=n, device=dev,
                                             dtype=torch.float32)
    gen = torch.Generator(dev).manual_seed(seed)
    pool = torch.empty((pool_size, N_AGENTS, ACT_DIM, n), dtype=torch.float32, device=dev)
    pool.uniform_(-1.0, 1.0, generator=gen)
    packed = pool.transpose(2, 3)
    env.reset()
    k = [0]

    host = []

    def run(m):
        for _ in range(m):
            h0 = time.perf_counter()
            _, _, dones, _ = env.step(packed[k[0] % pool_size])
            k[0] += 1
            if dones["__all__"]:
                env.reset()
            host.append(time.perf_counter() - h0)
    # as the headline: one whole episode first (every step's launch state built
    # once, cached across episodes), then collect, then the warmup steps
    run(warmup)
    while env.episode_step != 0:
        run(1)
    gc.collect()
    gc.freeze()
    run(warmup)
    torch.cuda.synchronize()
    del host[:]
    t0 = time.perf_counter()
    run(steps)
    t_host = time.perf_counter()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    host_us = {"sum": sum(host) * 1e6, "max": max(host) * 1e6, "argmax": host.index(max(host)),
               "sync_wait": (time.perf_counter() - t_host) * 1e6}
    # kernel durations in a separate pass (every launch event-timed), as the headline's
    tot, cnt = timed_pass(run, 64)
    a_us = tot[0] / cnt[0] * 1e3 if cnt[0] else None
    p_us = tot[1] / cnt[1] * 1e3 if cnt[1] else None
    out = {"dtype": "f32 storage, f64 arithmetic", "value": N_AGENTS * n * steps / dt,
           "unit": "agent-env-steps/s", "ms_per_step": dt / steps * 1e3, "steps": steps,
           "host_us": host_us,
           "parity": "tests/test_gpu_f32.py::test_c4_f32_one_step_parity[%s] (one step = fp64 result "
                     "rounded once) and ::test_c4_f32_episode_within_bound[%s] (episode within 1e-3 rel "
                     "of fp64), both on this variant's kernels (pgw_coord_step_f32: %s)"
                     % (conv, conv, "k_coord_pf_od<14, pgw_coord_buffers_f32>" if conv == "opendss"
                        else "k_coord_pf<14,true,false,false, pgw_coord_buffers_f32>"),
           "k_coord_agents_std": {"avg_us": a_us, "bytes_per_launch": AGENT_BYTES_F32 * N_AGENTS * n,
                                  "achieved": (AGENT_BYTES_F32 * N_AGENTS * n / (a_us * 1e-6) / 1e9
                                               if a_us else None),
                                  "peak": HBM_PEAK_GBS, "unit": "GB/s"},
           "k_coord_pf_avg_us": p_us,
           "kernel_timing": "every launch of a separate 64-step pass after the timed region"}
    if a_us:
        out["k_coord_agents_std"]["frac"] = out["k_coord_agents_std"]["achieved"] / HBM_PEAK_GBS
    return out


def timed_pass(run, steps):
    """Kernel durations: `steps` more steps with every launch bracketed by HIP
    events on its own stream (pgw_timing_*); returns (total ms, launches) per
    PGW_T_* slot.  Never inside a timed region: an event-bracketed launch costs
    ~10 us of step time."""
    from powergridworld_amd import _lib
    _lib.check(_lib.lib().pgw_timing_start(1))
    run(steps)
    torch.cuda.synchronize()
    tot = (_lib.C.c_double * len(KERNELS))()
    cnt = (_lib.C.c_int64 * len(KERNELS))()
    _lib.check(_lib.lib().pgw_timing_stop(tot, cnt))
    return tot, cnt


def pf_variant(conv, n, steps, warmup, pool, dev, od_table=True):
    """The same C4 workload (same action pool) with the other power-flow stopping
    rule on the fused step: OpenDSS's snap solve (the reference's,
    opendss.py:131-135; pgw_coord_step + k_coord_pf_od) or the exact fixed point
    (k_coord_pf + its predictor).  Reported beside the headline."""
    from powergridworld_amd.scenarios.coordinated import (CoordinatedMultiBuildingControlEnv,
                                                          make_c4_config)
    env = CoordinatedMultiBuildingControlEnv(**make_c4_config(pf_convergence=conv), num_envs=n,
                                             device=dev, fused=True)
    env.pf_solver.od_table = bool(od_table)
    env.set_pf_list(env._one_launch_ok())           # (the one-launch step needs the table)
    P = pool.shape[0]
    env.reset()
    k = [0]

    def run(m):
        for _ in range(m):
            _, _, dones, _ = env.step(pool[k[0] % P])
            k[0] += 1
            if dones["__all__"]:
                env.reset()
    run(warmup)
    gc.collect()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tot, cnt = timed_pass(run, 64)
    it = env.pf_solver.iterations.abs().double()
    p_us = tot[1] / cnt[1] * 1e3 if cnt[1] else None
    table = conv == "opendss" and env.pf_solver.od_table
    out = {"pf_convergence": conv, "od_table": table, "value": N_AGENTS * n * steps / dt, "unit": "agent-env-steps/s",
           "ms_per_step": dt / steps * 1e3, "steps": steps, "pf_iterations_mean": float(it.mean()),
           "pf_iterations_max": int(it.max()),
           "k_coord_agents_std_avg_us": tot[0] / cnt[0] * 1e3 if cnt[0] else None,
           "pf_kernel": {"name": (PF_KERNEL_NAME[conv] if env.pf_solver._od_fast or conv == "exact"
                                  else "k_pf_general"), "avg_us": p_us}}
    if conv == "opendss" and not table:
        out["note"] = ("OpenDSS's rule with every env's snap solve run (od_table=False): the reference's rule "
                       "without the per-hour response table (k_coord_agents_std + k_coord_pf_od)")
    if p_us:
        out["pf_kernel"].update(pf_roofline(conv, p_us, float(it.mean()), n, table))
    del env
    return out


def graph_variant(env, packed, steps, warmup_episodes=1, S=8):
    """The headline's env and action pool with the fused step captured S steps
    per hipGraph (MultiAgentEnv.capture_step: one graph per episode position,
    the pool entry of each step bound at capture); the tail of an episode
    (fewer than S steps left) and the resets run eagerly.  Bit-identical to the
    eager step (tests/test_gpu_graph.py::test_c4_graph8_equals_eager_across_
    episodes).  Reported beside the eager headline, never as it."""
    P = packed.shape[0]
    graph = env.capture_step(lambda k: [packed[(k + i) % P] for i in range(S)], steps=S)
    env.reset()

    def run(m):
        done_steps, calls = 0, 0
        while done_steps < m:
            k, last = env.episode_step, env._episode_last_step()
            if k + S <= last:
                _, _, d, _ = graph()
                done_steps += S
                calls += 1
            else:
                _, _, d, _ = env.step(packed[k % P])
                done_steps += 1
            if d["__all__"]:
                env.reset()
        return done_steps, calls
    t0 = time.perf_counter()
    run(warmup_episodes * 286)                      # every position's graph captured
    capture_s = time.perf_counter() - t0
    gc.collect()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done_steps, calls = run(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n_graphs = len(graph._pos)
    graph.release()                  # (not at a later garbage collection, inside another variant's timing)
    return {"value": N_AGENTS * env.num_envs * done_steps / dt, "unit": "agent-env-steps/s",
            "ms_per_step": dt / done_steps * 1e3, "steps": done_steps, "graph_calls": calls,
            "graphs": n_graphs, "warmup_capture_s": capture_s,
            "note": "S=%d steps per hipGraph launch (one graph per episode position and list parity, captured "
                    "in a warm-up episode), episode tails and resets eager; same env, state and action pool as "
                    "the headline, bit-identical outputs" % S}


def _oracle_leg(job):
    """One process of the CPU baseline: the oracle, 1 thread, on its own envs."""
    envs, steps, seed = job
    from threadpoolctl import threadpool_limits
    from oracle.ma_oracle import CoordinatedOracle
    rng = np.random.default_rng(seed)
    with threadpool_limits(limits=1):
        orc = CoordinatedOracle(envs)
        orc.reset(rng.uniform(3, 50, (N_AGENTS, envs)))
        acts = [rng.uniform(-1, 1, (N_AGENTS, envs, ACT_DIM)) for _ in range(steps)]
        t0 = time.perf_counter()
        for a in acts:
            orc.step(a)
        return time.perf_counter() - t0


def cpu_baseline(envs, steps, procs):
    """The oracle (batched NumPy port of the reference step path + PF) on the
    host: 1 process, then `procs` forked processes on independent env shards
    (k = 1 and k = 8).  Runs before any GPU call, so the forks
    never copy a GPU context.  value = the k-process aggregate."""
    import multiprocessing as mp
    units = N_AGENTS * envs * steps
    t1 = _oracle_leg((envs, steps, 0))
    with mp.get_context("fork").Pool(procs) as pool:
        tk = pool.map(_oracle_leg, [(envs, steps, 1 + r) for r in range(procs)])
    out = {"value": procs * units / max(tk), "unit": "agent-env-steps/s", "cores": procs,
           "kind": "port",
           "sample": "oracle/ma_oracle.CoordinatedOracle (batched NumPy fp64 port of the reference "
                     "step path + PF), %d processes x %d envs x %d steps, 1 thread each, slowest "
                     "%.1f s" % (procs, envs, steps, max(tk)),
           "per_core": {"value": units / t1, "cores": 1, "sample": "1 process, %d envs x %d steps, "
                                                                  "%.1f s" % (envs, steps, t1)}}
    p = os.path.join(REPO, "profiles", "ref_cpu_loop.json")
    if os.path.exists(p):
        with open(p) as f:
            ref = json.load(f)
        out["reference_loop"] = {
            "note": "the reference's own Python loop (stub PF), timed by tools/ref_cpu_loop.py in the "
                    "build container; it cannot run on the GPU host",
            "host": ref.get("host"),
            "rows": [{"cores": r["cores"], "value": r["value"]} for r in ref.get("rows", [])],
            "survey_probe": [{"cores": 1, "value": 781.0}, {"cores": 8, "value": 5948.0}]}
    return out


def stream_copy_gbs(dev, nbytes=1 << 30, reps=20):
    """Measured HBM ceiling of this run: a device-to-device copy of `nbytes`
    (read + write = 2 x nbytes per copy) -- the library's 16-B-per-lane
    nontemporal copy kernel (pgw_stream_copy) and torch's copy_, each timed with
    events on the current stream; returns both in GB/s."""
    from powergridworld_amd import _lib
    a = torch.empty(nbytes // 8, dtype=torch.float64, device=dev).fill_(1.0)
    b = torch.empty_like(a)
    ms = _lib.C.c_float()
    _lib.check(_lib.lib().pgw_stream_copy(a.data_ptr(), b.data_ptr(), nbytes, reps, _lib.C.byref(ms),
                                          _lib.stream_ptr(dev)))
    kernel_gbs = 2 * nbytes / (ms.value * 1e-3) / 1e9
    for _ in range(3):
        b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    torch_gbs = 2 * nbytes / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9
    del a, b
    return kernel_gbs, torch_gbs


def load_traffic():
    """HBM bytes per launch from the committed PMC summary (tools/gpu/pmc_traffic.py)
    and, per kernel, the PMC run it came from (profiles/<round>/pmc_<run>.txt)."""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(p):
        with open(p) as f:
            d = json.load(f)
        return d.get("bytes_per_launch", {}), d.get("runs", {})
    return {}, {}


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(args):
    """--gpus N started without torchrun: run torch.distributed.run with N ranks
    as a CHILD process (never exec: nothing here has touched the GPU yet) and
    return its exit code.  Under torchrun, WORLD_SIZE must equal --gpus."""
    under = "WORLD_SIZE" in os.environ or "LOCAL_RANK" in os.environ
    if under:
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if world != args.gpus:
            sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d (one rank per GPU)" % (args.gpus, world))
        return None
    if args.gpus <= 1:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % args.gpus, "--master-addr=127.0.0.1",
           "--master-port=%d" % _free_port(), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    from powergridworld_amd import distributed as pgd
    rank, local, world = pgd.env_rank()
    dist = world > 1
    if args.cpu_baseline_only:
        print(json.dumps(cpu_baseline(args.cpu_sample_envs, args.cpu_sample_steps, args.cpu_procs)))
        return
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        # a child process, started before this one touches the GPU: the oracle's
        # imports and garbage never enter the timed process
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-baseline-only",
                            "--cpu-sample-envs", str(args.cpu_sample_envs), "--cpu-sample-steps",
                            str(args.cpu_sample_steps), "--cpu-procs", str(args.cpu_procs)],
                           stdout=subprocess.PIPE, check=True)
        cpu = json.loads(r.stdout.decode().strip().splitlines()[-1])
    # PGW_BENCH_REHEARSE=1: rehearse N ranks on fewer GPUs (ranks share devices
    # round-robin, collectives on gloo) -- a correctness check of the N>1 path,
    # never a measurement
    rehearse = os.environ.get("PGW_BENCH_REHEARSE") == "1"
    dev = torch.device("cuda", local % torch.cuda.device_count() if rehearse else local)
    torch.cuda.set_device(dev)
    pgd.init("gloo" if rehearse else "nccl", dev)
    if dist:
        import torch.distributed as tdist

    from powergridworld_amd.scenarios.coordinated import (CoordinatedMultiBuildingControlEnv,
                                                          make_c4_config)
    n = args.batch
    conv = args.pf_convergence
    env = CoordinatedMultiBuildingControlEnv(**make_c4_config(pf_convergence=conv), num_envs=n, device=dev,
                                             fused=True)
    if conv == "opendss" and not env.pf_solver._od_fast:
        raise RuntimeError("bench.py: the C4 feeder did not select the fast OpenDSS-rule kernel")
    env.set_pf_list(args.pf_split == "on")
    for i, agent in enumerate(env.agents):         # per-rank seed offset
        agent.env_dict["storage"].seed(pgd.rank_seed(0, rank, i))
    gen = torch.Generator(dev).manual_seed(pgd.rank_seed(0, rank))     # seed 0 at rank 0
    P = args.action_pool
    pool = torch.empty((P, N_AGENTS, ACT_DIM, n), dtype=torch.float64, device=dev)
    pool.uniform_(-1.0, 1.0, generator=gen)
    packed = pool.transpose(2, 3)                  # [P, agents, N, act_dim] view, env-minor

    step_count = 0
    host_t = []                                    # per-step host time of the last run() (diagnostics)

    def run(k):
        nonlocal step_count
        del host_t[:]
        for _ in range(k):
            h0 = time.perf_counter()
            _, _, dones, _ = env.step(packed[step_count % P])
            step_count += 1
            if dones["__all__"]:
                env.reset()
            host_t.append(time.perf_counter() - h0)

    from powergridworld_amd import _lib
    # the measured HBM ceiling of this box (device copy) -- also brings the GPU
    # out of its idle clocks after the host-only CPU baseline, before warmup
    copy_gbs, torch_copy_gbs = stream_copy_gbs(dev, reps=100)
    # one cold episode: the env's FIRST reset() -- the
    # power flow's per-hour tables built on the device (first-iteration tables,
    # the response table with its certificates, node records) -- and the
    # episode's steps, the first launches of every kernel included; then the
    # reset that starts the warm runs (not timed)
    torch.cuda.synchronize()
    c0 = time.perf_counter()
    env.reset()
    torch.cuda.synchronize()
    cold_reset = time.perf_counter() - c0
    cold_steps = 0
    while True:
        _, _, dones, _ = env.step(packed[step_count % P])
        step_count += 1
        cold_steps += 1
        if dones["__all__"]:
            break
    torch.cuda.synchronize()
    cold_total = pgd.max_over_ranks(time.perf_counter() - c0, dev)
    env.reset()
    # no garbage pending in the timed region -- collected BEFORE the warmup: the
    # first env.step after a gc.collect() costs ~120 us more host time (cold
    # caches), +6 us/step on a 20-step region (tools/gpu/short_region.py,
    # profiles/r02/short_region.txt); the warmup steps absorb it
    gc.collect()
    gc.freeze()
    run(args.warmup)
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    t_issued = time.perf_counter()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    host_region = {"issue_us": (t_issued - t0) * 1e6, "sync_wait_us": (time.perf_counter() - t_issued) * 1e6,
                   "step_max_us": max(host_t) * 1e6, "step_max_at": host_t.index(max(host_t)),
                   "step_median_us": sorted(host_t)[len(host_t) // 2] * 1e6,
                   "note": "host side of the timed region on rank 0: time to issue the steps, then the wait for "
                           "the GPU; the slowest step's host time and its index"}
    elapsed = pgd.max_over_ranks(elapsed, dev)
    # kernel durations: a second pass right after the timed region, every launch
    # bracketed by HIP events on its own stream.  Kept out of `value`'s region:
    # an event-bracketed launch costs ~10 us of extra step time (measured: the
    # driver-shaped 20-step run went 36 -> 44 us/step with every 2nd launch timed).
    # (a whole episode by default, whatever --steps: the one-launch step's
    # duration varies with the envs its table leaves to the inline solve --
    # rocprof 18.8-42.9 us per launch, r06k -- so a 20-launch mean is noise)
    time_steps = max(8, args.time_steps)
    tot, cnt = timed_pass(run, time_steps)
    # the PF iteration counts of the last timed-pass step (before the episode
    # pass below, which ends with a reset whose cold solve would overwrite them)
    iters_last = env.pf_solver.iterations.clone()
    unconverged = env.pf_solver.unconverged()
    # one whole episode: from the first step after a reset through
    # its last step AND the reset that follows (per-episode reset kernels, the
    # predictor-table solves of the next hours), no events; reported beside the
    # driver's region, which is shorter than an episode
    while True:
        _, _, dones, _ = env.step(packed[step_count % P])
        step_count += 1
        if dones["__all__"]:
            env.reset()
            break
    torch.cuda.synchronize()
    ep0, ep_steps = time.perf_counter(), 0
    while True:
        _, _, dones, _ = env.step(packed[step_count % P])
        step_count += 1
        ep_steps += 1
        if dones["__all__"]:
            env.reset()
            break
    torch.cuda.synchronize()
    ep_elapsed = pgd.max_over_ranks(time.perf_counter() - ep0, dev)
    # per-env statistics of the episode's last step, all-gathered in global env
    # order once per episode, outside every timed region (RCCL at N>1)
    ep_stats = pgd.gather_episode_stats(torch.stack(
        [iters_last.double(), env.pf_solver.get_bus_voltage_by_name("675c").double()], 1))
    total_envs = n * world
    value = N_AGENTS * total_envs * args.steps / elapsed
    if rank == 0:
        avg_us = {KERNELS[k]: (tot[k] / cnt[k] * 1e3 if cnt[k] else None) for k in range(len(KERNELS))}
        it = iters_last.abs().double()
        mean_it, max_it = float(it.mean()), int(it.max())
        # the PF runs one wave (64 envs) per SIMD: its time follows the slowest
        # wave, so report how many waves need 1, 2, ... iterations
        wenv = 64                                                             # envs per PF wave
        wmax = iters_last.abs()[: (n // wenv) * wenv].view(-1, wenv).max(1).values
        wave_hist = {int(k): int(v) for k, v in zip(*torch.unique(wmax, return_counts=True))}
        traffic, traffic_runs = load_traffic()
        kernels = {}
        a_us, p_us = avg_us[KERNELS[0]], avg_us[KERNELS[1]]
        table = conv == "opendss" and env.pf_solver.od_table
        split = table and bool(env._fused.get("od_on"))
        ak = "k_coord_step_od" if split else "k_coord_agents_std"
        a_bytes = STEP_OD_ENV_BYTES * n if split else AGENT_BYTES * N_AGENTS * n
        if a_us:
            gbs = a_bytes / (a_us * 1e-6) / 1e9
            kernels[ak] = {"avg_us": a_us, "timed_launches": cnt[0], "bound": "hbm",
                           "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": gbs / HBM_PEAK_GBS, "bytes_per_launch": a_bytes,
                           "traffic": traffic.get(ak), "traffic_run": traffic_runs.get(ak)}
            if split:
                kernels[ak]["note"] = ("the whole step in one launch: the 5 agents' steps, the power flow's "
                                       "response-table lookup (node records) and the snap solve of the envs the "
                                       "table leaves (the lookup wave, od_wave_solve): %d B per env (agents 5 x %d "
                                       "+ V675.3, violation, iteration count)" % (STEP_OD_ENV_BYTES, AGENT_BYTES))
                kernels[ak]["solved_inline_last_step"] = int(
                    env._fused["od_count"][env._fused["bufs"].od_parity & 1])
        if split and table and a_us:
            kernels[ak]["response_table"] = table_stats(env)
        if p_us:
            pk = "k_coord_pf_od_list<14>" if split else PF_KERNEL_NAME[conv]
            kernels[pk] = {"avg_us": p_us, "timed_launches": cnt[1],
                           "note": ("the hour's response table serves every env whose kW lies in a fitted "
                                    "piece, the snap solve (fp64 VALU DPP FMAs) the rest" if table else
                                    "fp64 VALU DPP FMAs, no MFMA (MI355X fp64 vector peak = matrix peak); "
                                    "issue-bound, one wave per SIMD at 65,536 envs"),
                           "traffic": traffic.get(pk), "traffic_run": traffic_runs.get(pk)}
            if not split:
                kernels[pk]["hbm_gbs"] = PF_BYTES * n / (p_us * 1e-6) / 1e9
            kernels[pk].update(pf_roofline(conv, p_us, mean_it, n, table, split))
            if table:
                kernels[pk]["response_table"] = table_stats(env)
        if avg_us[KERNELS[2]]:
            kernels[KERNELS[2]] = {"avg_us": avg_us[KERNELS[2]], "timed_launches": cnt[2],
                                   "note": "reset power flow + predictor tables (24 h x 3201 grid points "
                                           "per launch), all k_pf_solve variants"}
        for k in kernels.values():
            if k.get("unit") == "GB/s":
                k["frac_measured_copy"] = k["achieved"] / copy_gbs
        dom = max((k for k in kernels if "achieved" in kernels[k]), key=lambda k: kernels[k]["avg_us"])
        d = kernels[dom]
        roof = {"kernel": dom, "bound": d["bound"], "achieved": d["achieved"], "peak": d["peak"],
                "unit": d["unit"], "frac": d["frac"], "traffic": d["traffic"],
                "traffic_run": d.get("traffic_run"),
                "avg_launch_us": d["avg_us"], "timed_launches": d["timed_launches"]}
        if d["unit"] == "GB/s":
            roof["peak_measured_copy"] = copy_gbs
            roof["frac_measured_copy"] = d["achieved"] / copy_gbs
        step_bytes = (AGENT_BYTES * N_AGENTS + 8) * n      # 1,568 B per C4 env-step
        step_gbs = step_bytes / (elapsed / args.steps) / 1e9
        step = {"bytes_per_step": step_bytes, "achieved": step_gbs, "unit": "GB/s",
                "frac": step_gbs / HBM_PEAK_GBS, "frac_measured_copy": step_gbs / copy_gbs,
                "note": "algorithmic HBM bytes of the whole step (SURVEY 8(d): agents 312 B x 5 + "
                        "V675.3 8 B per env) / ms_per_step, per GPU"}
        out = {
            "metric": "agent-env-steps/sec at batch 65536, 5-agent scenario, 1/2/4/8 MI355X",
            "value": value,
            "unit": "agent-env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "ms_per_step_episode": ep_elapsed / ep_steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded uniform actions pre-generated on device, synthetic "
                    "exogenous building data, IEEE-13 feeder + 8760-h loadshape)",
            "config": {"workload": "C4: 5-agent coordinated buildings (building+PV+storage) "
                                   "+ IEEE-13 power flow + voltage-violation reward",
                       "pf_convergence": conv,
                       "batch_per_gpu": n, "global_batch": total_envs, "episode_steps": 286,
                       "parallelism": "env-sharded x%d (no collective on the step path)" % world},
            "roofline": roof,
            "step_hbm": step,
            "stream_copy_gbs": copy_gbs,
            "stream_copy": {"kernel_gbs": copy_gbs, "torch_copy_gbs": torch_copy_gbs,
                            "note": "1 GiB device copy, 2 x bytes per copy; kernel = pgw_stream_copy "
                                    "(16 B/lane, nontemporal), the measured peak used for frac_measured_copy"},
            "kernels": kernels,
            "kernel_timing": {"steps": time_steps, "every_launch": True,
                              "note": "HIP events around every launch of a separate pass of "
                                      "`steps` steps right after the timed region (not inside it)"},
            "pf_iterations": {"mean": mean_it, "max": max_it, "wave_max_hist": wave_hist,
                              "unconverged_envs": unconverged},
            "episode_cold": {"steps": cold_steps, "ms": cold_total * 1e3, "reset_ms": cold_reset * 1e3,
                             "ms_per_step": cold_total / cold_steps * 1e3,
                             "value": N_AGENTS * total_envs * cold_steps / cold_total,
                             "pf_table_build_s": env.pf_solver.od_resp_stats.get("build_s"),
                             "note": "the env's first reset() (the power flow's per-hour tables built and "
                                     "certified on the device) plus the whole first episode, first launches "
                                     "included, no events"},
            "host_region": host_region,
            "episode": {"steps": ep_steps, "ms_per_step": ep_elapsed / ep_steps * 1e3,
                        "gathered_env_stats": int(ep_stats.shape[0]),
                        "value": N_AGENTS * total_envs * ep_steps / ep_elapsed,
                        "note": "one whole episode after the timed region: its %d steps and the "
                                "env.reset() that ends it (reset kernels, predictor tables of the "
                                "next hours), no events" % ep_steps},
        }
        if world == 1 and not args.no_variants:
            other = "exact" if conv == "opendss" else "opendss"
            out["variants"] = {"graph8": graph_variant(env, packed, args.steps),
                               "f32": f32_variant(conv, n, min(args.steps, 286), args.warmup, P,
                                                  pgd.rank_seed(0, rank), dev),
                               other + "_pf": pf_variant(other, n, min(args.steps, 286), args.warmup, packed,
                                                         dev)}
            if conv == "opendss":
                out["variants"]["opendss_no_table"] = pf_variant("opendss", n, min(args.steps, 286), args.warmup,
                                                                 packed, dev, od_table=False)
        if cpu is not None:
            out["cpu_baseline"] = cpu
        print(json.dumps(out))
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
