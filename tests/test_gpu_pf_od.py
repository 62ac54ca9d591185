"""OpenDSS's snap-solve rule on the fast one-lane-per-env kernels
(pgw_pf_tables.od; csrc/pgw_pf.hip k_pf_solve_od / k_coord_pf_od): the C4
shape (IEEE-13, one controllable load).  Needs an MI355X.

PF parity is unpinned (no OpenDSS in this image): the results are
checked against the oracle's NumPy restatement of OpenDSS's snap solve,
oracle/pf_oracle.py Feeder.snap_opendss (the loads' Yeq in Y at the DSS
file's kW, direct-solution start, every node's magnitude change <= 1e-4 from
iteration 2, at most 15) -- equal iteration counts for every env, every node
within 1e-9 rel -- and against the general kernel's implementation of the same
rule.  The fast kernels evaluate only some check rows and bound the others;
the tests pin that this never changes a result: bounded (fast) == every row
(full) == every wave re-run, bit for bit.
"""
import os

import numpy as np
import pandas as pd
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
HERE = os.path.dirname(os.path.abspath(__file__))
IEEE13 = "ieee_13_dss/IEEE13Nodeckt.dss"
SHAPE = "ieee_13_dss/annual_hourly_load_profile.csv"
TIMES = [pd.Timestamp("08-12-2021 %02d:10:00" % h) for h in (3, 11, 17, 20)]


def _solver(**kw):
    from powergridworld_amd.distribution_system.opendss import OpenDSSSolver
    return OpenDSSSolver(IEEE13, SHAPE, device=DEV, system_load_rescale_factor=1.2, convergence="opendss", **kw)


def _loads(K, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in TIMES:
        p = rng.uniform(-400.0, 900.0, K)
        q = rng.uniform(-0.3, 0.5, K) * np.abs(p)
        out.append((p, q))
    return out


def _solve_all(s, loads):
    """[T, n_nodes, K] pu and [T, K] iterations of s over TIMES."""
    v, it = [], []
    for t, (p, q) in zip(TIMES, loads):
        s.calculate_power_flow({"675c": torch.tensor(p, device=DEV)}, {"675c": torch.tensor(q, device=DEV)},
                               current_time=t)
        bv = s.get_bus_voltages()
        v.append(torch.stack([bv[nm] for nm in s.feeder.node_names]).clone())
        it.append(s.iterations.clone())
    torch.cuda.synchronize()
    return torch.stack(v), torch.stack(it)


def test_od_fast_kernel_selected():
    s = _solver(num_envs=8)
    assert s._od_fast and not s.general and s.M == 14
    od = s._od_proto
    assert 0 < od.n_rep < od.n_rows <= 32 and od.min_iter == 2 and od.tol == 1e-4
    # every node is covered exactly once: an element's terminal or a check row
    elem = {s.feeder.node_names[s.feeder.elem_p[k]] for k in range(s.feeder.m) if s.feeder.elem_q[k] < 0}
    assert sorted(elem | set(s._od_rows)) == sorted(s.feeder.node_names) and not (elem & set(s._od_rows))
    s.set_controllable_loads(["675a", "675c"])           # two slots: the general kernel
    assert s.general and not s._od_fast
    g = _solver(num_envs=8, general=True)
    assert g.general and not g._od_fast


def test_od_ieee13_vs_oracle_and_general_kernel():
    """The fast kernel's stopped iterate equals the oracle's restatement of
    OpenDSS's snap solve (same iterations, every node within 1e-9 rel) and the
    general kernel's (same iterations, 1e-11 rel)."""
    from oracle.pf_oracle import BatchedPF
    K = 4096
    loads = _loads(K, 2)
    v, it = _solve_all(_solver(num_envs=K), loads)
    vg, itg = _solve_all(_solver(num_envs=K, general=True), loads)
    assert torch.equal(it, itg)
    torch.testing.assert_close(v, vg, rtol=1e-11, atol=0)
    o = BatchedPF(system_load_rescale_factor=1.2)
    f = o.feeder
    for i, (t, (p, q)) in enumerate(zip(TIMES, loads)):
        kw, kvar = o.loads(t, {"675c": p}, {"675c": q}, K=K)
        V, oit = f.snap_opendss(kw, kvar, f.base_kw, f.base_kvar)
        np.testing.assert_array_equal(it[i].cpu().numpy(), oit)
        np.testing.assert_allclose(v[i].cpu().numpy().T, f.pu(V), rtol=1e-9, atol=0)
    assert set(np.unique(it.cpu().numpy())) <= set(range(2, 16))


def test_od_bounded_rows_equal_every_row_and_rerun():
    """The bounded check rows never change a result: the fast kernel equals
    the same solve with every row evaluated (n_rep = n_rows), and a solve whose
    bounds can never decide (every wave re-runs with every row) -- bit for bit,
    iteration counts included."""
    K = 4096
    loads = _loads(K, 3)
    ref = _solve_all(_solver(num_envs=K), loads)
    # also: every wave's rows as row groups (sparse_envs < 0) and every
    # tested env's rows one env at a time (64), with and without bounds that
    # decide -- the transposed evaluation (od_rows_sparse) against the DPP row
    # groups, bit for bit
    for change in (dict(n_rep=None), dict(gsrc=1e9), dict(sparse_envs=-1), dict(sparse_envs=64),
                   dict(sparse_envs=64, gsrc=1e9), dict(sparse_envs=-1, gsrc=1e9)):
        s = _solver(num_envs=K)
        if change.get("n_rep", 0) is None:
            s._od_proto.n_rep = s._od_proto.n_rows
        if "gsrc" in change:
            s._od_proto.gsrc = change["gsrc"]
        if "sparse_envs" in change:
            s._od_proto.sparse_envs = change["sparse_envs"]
        s._tables_cache.clear()
        got = _solve_all(s, loads)
        assert torch.equal(got[1], ref[1]), change
        assert torch.equal(got[0], ref[0]), change


def test_od_c4_fused_equals_generic_and_oracle():
    """C4 with convergence="opendss" on the fast kernels: the fused step
    (pgw_coord_step + k_coord_pf_od) is bit-identical to the generic path
    (component kernels + k_pf_solve_od) and matches the NumPy C4 oracle with
    OpenDSS's snap semantics: rewards, violation, V675.3, iteration counts."""
    from oracle.ma_oracle import CoordinatedOracle
    from oracle.pf_oracle import BatchedPF
    from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config
    n = 256
    fused, generic = [CoordinatedMultiBuildingControlEnv(**make_c4_config(pf_convergence="opendss"), num_envs=n,
                                                         device=DEV, fused=f) for f in (True, False)]
    assert fused._fused is not None and fused._fused["kernel"] == "pgw_coord_step" and fused.pf_solver._od_fast
    assert generic._fused is None and generic.pf_solver._od_fast
    rng = np.random.default_rng(11)
    init = rng.uniform(5.0, 45.0, size=(5, n))
    for env in (fused, generic):
        env.reset()
        for ai, agent in enumerate(env.agents):
            agent.env_dict["storage"].reset(init_storage=torch.tensor(init[ai], device=DEV))
        env.load_component_state()
    ora = CoordinatedOracle(n)
    ora.pf = BatchedPF(system_load_rescale_factor=1.2, semantics="opendss")
    ora.reset(init)
    for t in range(40):
        act = rng.uniform(-1, 1, size=(5, n, 8))
        a_t = torch.tensor(act, device=DEV)
        of, rf, _, mf = fused.step(a_t)
        og, rg, _, mg = generic.step({a.name: {"building": a_t[i, :, :6], "pv": a_t[i, :, 6:7],
                                               "storage": a_t[i, :, 7:8]} for i, a in enumerate(generic.agents)})
        o_obs, o_rew, o_vv = ora.step(act)
        torch.cuda.synchronize()
        assert torch.equal(mf["voltage_violation"], mg["voltage_violation"])
        for a in fused.agents:
            assert torch.equal(rf[a.name], rg[a.name])
        assert torch.equal(fused.pf_solver.iterations, generic.pf_solver.iterations)
        np.testing.assert_allclose(fused.packed_obs().cpu().numpy(), o_obs, rtol=1e-9, atol=1e-9)
        r = np.stack([rf[a.name].cpu().numpy() for a in fused.agents])
        np.testing.assert_allclose(r, o_rew, rtol=1e-7, atol=1e-7)
        np.testing.assert_allclose(fused.pf_solver.get_bus_voltage_by_name("675c").cpu().numpy(), ora.v,
                                   rtol=1e-10, atol=0)
        np.testing.assert_array_equal(fused.pf_solver.iterations.cpu().numpy(), ora.pf.last_iters)
    v_f, v_g = fused.voltages, generic.voltages
    for nm in ("632.1", "671.2", "652.1", "675.3"):
        assert torch.equal(v_f[nm], v_g[nm])


def test_od_c4_two_episodes_tiled_full_batch():
    """The BASELINE batch (65,536 envs, fused, OpenDSS rule) on the
    c4_two_episodes golden action streams tiled over the batch, against the C4
    oracle with OpenDSS's snap solve run on the golden envs: every env's
    iteration count equal at every step of both episodes, V675.3 within 1e-10
    rel, violation within 1e-11, rewards within 1e-7 (errors accumulated on the
    device, one check per episode)."""
    from oracle.ma_oracle import CoordinatedOracle
    from oracle.pf_oracle import BatchedPF
    from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config
    g = np.load(os.path.join(HERE, "golden", "c4_two_episodes.npz"))
    E, Tn, NA, K, _ = g["actions"].shape
    n = 65536
    idx = torch.arange(n, device=DEV) % K
    env = CoordinatedMultiBuildingControlEnv(**make_c4_config(pf_convergence="opendss"), num_envs=n, device=DEV,
                                             fused=True)
    assert env._fused["kernel"] == "pgw_coord_step" and env.pf_solver._od_fast
    T = lambda a: torch.tensor(np.asarray(a), dtype=torch.float64, device=DEV)
    acts = T(g["actions"])[:, :, :, idx]
    ora = CoordinatedOracle(K)
    ora.pf = BatchedPF(system_load_rescale_factor=1.2, semantics="opendss")
    hist = {2: 0, 3: 0, 4: 0, 5: 0}
    for e in range(E):
        err = torch.zeros(4, dtype=torch.float64, device=DEV)
        env.reset()
        for a, agent in enumerate(env.agents):
            agent.env_dict["storage"].reset(init_storage=T(g["init_storage"][e, a])[idx])
        ora.reset(g["init_storage"][e])
        for t in range(Tn):
            _, rew, dones, meta = env.step(acts[e, t])
            _, o_rew, o_vv = ora.step(g["actions"][e, t])
            want_it = T(ora.pf.last_iters.astype(np.float64))[idx]
            for i in np.unique(ora.pf.last_iters):
                hist[int(i)] = hist.get(int(i), 0) + 1
            r = torch.stack([rew[a.name] for a in env.agents])
            wr = T(o_rew)[:, idx]
            err[0] = torch.maximum(err[0], ((r - wr).abs() / (1e-7 + 1e-7 * wr.abs())).max())
            err[1] = torch.maximum(err[1], (meta["voltage_violation"] - T(o_vv)[idx]).abs().max())
            v = env.pf_solver.get_bus_voltage_by_name("675c")
            err[2] = torch.maximum(err[2], ((v - T(ora.v)[idx]).abs() / T(ora.v)[idx]).max())
            err[3] = err[3] + (env.pf_solver.iterations.double() != want_it).sum()
            assert dones["__all__"] == bool(g["done"][e, t, 0])
        err = err.cpu().numpy()
        assert err[0] <= 1 and err[1] < 1e-11 and err[2] < 1e-10 and err[3] == 0, (e, err)
    assert hist[3] + hist[4] > 0, hist


# ------------------------------------------------------------------ response table (pgw_pf_od.resp)
def _served(s, hour, P):
    """The envs whose (P, Q = 0) the hour's response table serves: the kernels'
    lookup (od_resp_lookup) restated on the host from the downloaded records."""
    from powergridworld_amd import _lib
    idx = s._od_index[s._hour_key(hour)]
    recs = s._od_resp[idx].cpu().numpy()
    words = recs[:, 4].copy().view(np.int64)
    its, nxt = (words & 0xffffffff).astype(np.int64), words >> 32
    nseg = s.PREDICTOR_N - 1
    out = np.zeros(len(P), bool)
    g = (P - s.PREDICTOR_X0) * (1.0 / s.PREDICTOR_H)
    for e, (p, gg) in enumerate(zip(P, g)):
        if not (0.0 <= gg < nseg):
            continue
        r = int(gg)
        for _ in range(8):
            if recs[r, 0] <= p <= recs[r, 1]:
                out[e] = its[r] != 0
                break
            if nxt[r] < 0:
                break
            r = int(nxt[r])
    assert recs.shape[1] == _lib.od_rec(s.M)
    return out


def test_od_response_table_equals_solve():
    """The response table against every env solved (od_table=False) at the
    BASELINE batch, over the whole kW grid and right beside every breakpoint
    bracket (1e-9 .. 1e-3 kW off either end): the same iteration count for
    every env, every node within 1e-11 rel (the fit is checked at 2e-11 on the
    currents); the table serves all but the brackets' envs; the build's
    statistics are sane (no unresolved bracket, fit error within tolerance)."""
    K = 65536
    tab, sol = _solver(num_envs=K), _solver(num_envs=K, od_table=False)
    rng = np.random.default_rng(7)
    zero = torch.zeros(K, dtype=torch.float64, device=DEV)
    for t in TIMES:
        # builds the hour's tables (24 hours ahead) for the controllable slot
        tab.calculate_power_flow({"675c": zero}, None, current_time=t)
        hour = tab.hour_of(t)
        br = tab.od_resp_brackets[tab._od_index[tab._hour_key(hour)]]
        assert len(br) > 0
        near = np.concatenate([br[:, 0] - d for d in (1e-9, 1e-6, 1e-3)] + [br[:, 1] + d for d in (1e-9, 1e-6, 1e-3)]
                              + [0.5 * (br[:, 0] + br[:, 1])])
        P = np.concatenate([rng.uniform(-520.0, 1520.0, K - len(near)), near])
        v = []
        for s_ in (tab, sol):
            s_.calculate_power_flow({"675c": torch.tensor(P, device=DEV)}, None, current_time=t)
            bv = s_.get_bus_voltages()
            v.append((torch.stack([bv[nm] for nm in s_.feeder.node_names]).clone(), s_.iterations.clone()))
        torch.cuda.synchronize()
        (vt, it_t), (vs, it_s) = v
        assert torch.equal(it_t, it_s), int((it_t != it_s).sum())
        rel = ((vt - vs).abs() / vs.abs()).max().item()
        assert rel < 1e-11, rel
        served = _served(tab, hour, P)
        inside = (P >= tab.PREDICTOR_X0) & (P < tab.PREDICTOR_X0 + (tab.PREDICTOR_N - 1) * tab.PREDICTOR_H)
        assert served[: K - len(near)][inside[: K - len(near)]].mean() > 0.999
        assert not served[-len(br):].any()                # bracket midpoints: the solve
    st = tab.od_resp_stats
    assert st["unresolved_brackets"] == 0 and st["max_fit_err"] <= tab.OD_RESP_TOL, st
    assert st["pieces_left_to_solve"] <= 0.01 * st["pieces"], st


@pytest.mark.parametrize("scenario", ["c4", "het"])
def test_od_response_table_dense_every_hour(scenario):
    """The certified response table against every env solved, densely: all 24
    hours of the scenario's day, 64 points inside every one of the grid's 3 200
    segments of 0.625 kW (204 800 envs per hour, 4.9 M probes per scenario):
    the same iteration count at every point, every node within 1e-11 rel.  C4:
    rescale 1.2 on 2021-08-12 (make_c4_config); HET: rescale 0.65 on 2020-08-12
    (heterogeneous.make_env_config)."""
    rescale, day = {"c4": (1.2, "08-12-2021"), "het": (0.65, "08-12-2020")}[scenario]
    nseg, per = 3200, 64
    K = nseg * per
    from powergridworld_amd.distribution_system.opendss import OpenDSSSolver
    tab, sol = [OpenDSSSolver(IEEE13, SHAPE, device=DEV, system_load_rescale_factor=rescale, num_envs=K,
                              convergence="opendss", od_table=o) for o in (True, False)]
    x0, h = tab.PREDICTOR_X0, tab.PREDICTOR_H
    j = np.repeat(np.arange(nseg), per)
    P = x0 + h * (j + (np.tile(np.arange(per), nseg) + 0.5) / per)
    Pd = torch.tensor(P, device=DEV)
    worst, mism, served_n = 0.0, 0, 0
    for hr in range(24):
        t = pd.Timestamp("%s %02d:10:00" % (day, hr))
        res = []
        for s_ in (tab, sol):
            s_.calculate_power_flow({"675c": Pd}, None, current_time=t)
            bv = s_.get_bus_voltages()
            res.append((torch.stack([bv[nm] for nm in s_.feeder.node_names]), s_.iterations.clone()))
        (vt, it_t), (vs, it_s) = res
        mism += int((it_t != it_s).sum())
        worst = max(worst, ((vt - vs).abs() / vs.abs()).max().item())
        served_n += int(_served(tab, tab.hour_of(t), P).sum())
        del res, vt, vs
    st = tab.od_resp_stats
    print("dense %s: %d probes, %d iteration mismatches, worst node rel %.3e, served %.6f; table %s"
          % (scenario, 24 * K, mism, worst, served_n / (24 * K), st))
    assert mism == 0 and worst < 1e-11, (mism, worst)
    assert served_n > 0.999 * 24 * K
    assert st["certified"] and st["unresolved_brackets"] == 0, st


def test_od_response_table_bit_identical_paths():
    """The fused C4 step, the generic path and the all-node solve read the same
    table records with the same operations: fused == generic bit for bit over a
    stretch of an episode with the table serving, and the fused step with the
    table off (every env solved) equals the oracle as the table does."""
    from oracle.ma_oracle import CoordinatedOracle
    from oracle.pf_oracle import BatchedPF
    from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config
    n = 1024
    envs = [CoordinatedMultiBuildingControlEnv(**make_c4_config(), num_envs=n, device=DEV, fused=f)
            for f in (True, False, True)]
    envs[2].pf_solver.od_table = False
    rng = np.random.default_rng(13)
    init = rng.uniform(5.0, 45.0, size=(5, n))
    for env in envs:
        env.reset()
        for ai, agent in enumerate(env.agents):
            agent.env_dict["storage"].reset(init_storage=torch.tensor(init[ai], device=DEV))
    ora = CoordinatedOracle(n)
    ora.pf = BatchedPF(system_load_rescale_factor=1.2, semantics="opendss")
    ora.reset(init)
    for t in range(60):
        act = rng.uniform(-1, 1, size=(5, n, 8))
        a_t = torch.tensor(act, device=DEV)
        outs = [envs[0].step(a_t),
                envs[1].step({a.name: {"building": a_t[i, :, :6], "pv": a_t[i, :, 6:7], "storage": a_t[i, :, 7:8]}
                              for i, a in enumerate(envs[1].agents)}),
                envs[2].step(a_t)]
        _, o_rew, o_vv = ora.step(act)
        torch.cuda.synchronize()
        assert torch.equal(outs[0][3]["voltage_violation"], outs[1][3]["voltage_violation"])
        for a in envs[0].agents:
            assert torch.equal(outs[0][1][a.name], outs[1][1][a.name])
        for env in envs:
            np.testing.assert_array_equal(env.pf_solver.iterations.cpu().numpy(), ora.pf.last_iters)
            np.testing.assert_allclose(env.pf_solver.get_bus_voltage_by_name("675c").cpu().numpy(), ora.v,
                                       rtol=1e-10, atol=0)
    for nm in ("632.1", "671.2", "652.1", "675.3"):
        assert torch.equal(envs[0].voltages[nm], envs[1].voltages[nm])


def _unfit(solver, every):
    """Mark every `every`-th response record of the solver's tables unfit (k*
    = 0, the chain kept) in the response records and their node records: the
    envs in those pieces go to the solve."""
    from powergridworld_amd import _lib
    for tab, R in ((solver._od_resp, _lib.od_rec(solver.M)), (solver._od_vresp, _lib.OD_VREC)):
        w = tab.view(-1, R).view(torch.int64)[:, 4]
        sel = torch.arange(w.shape[0], device=w.device) % every == 0
        w[sel] = w[sel] & ~0xffffffff


@pytest.mark.parametrize("n,every,steps", [(4133, 0, 40), (4133, 3, 20), (4133, 1, 12), (66000, 1, 3)])
def test_od_split_step_bit_identical(n, every, steps):
    """The fused C4 step with the agents, the table lookup and the snap solve
    of the envs the table leaves in one launch (k_coord_step_od: the lookup
    wave's od_wave_solve, one env at a time; with PGW_STEP_LIST=1 the list form,
    those envs listed for k_coord_pf_od_list) against the two-kernel step
    (k_coord_agents_std + k_coord_pf_od): every output bit for bit -- with the
    table serving (every = 0), with a third of the records forced unfit and with
    all of them (every env solved by the wave solve; at 66 000 envs, 1 032
    blocks of 64 solves each) -- and the all-unfit case equal to the step
    without a table (od_table=False).  od_count counts the envs left to the
    solve in both forms."""
    from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config
    envs = [CoordinatedMultiBuildingControlEnv(**make_c4_config(), num_envs=n, device=DEV, fused=True)
            for _ in range(3)]
    envs[0].set_pf_list(True)
    envs[1].set_pf_list(False)
    envs[2].set_pf_list(False)
    envs[2].pf_solver.od_table = False
    rng = np.random.default_rng(17)
    init = torch.tensor(rng.uniform(5.0, 45.0, size=(5, n)), device=DEV)
    for env in envs:
        env.reset()
        for ai, agent in enumerate(env.agents):
            agent.env_dict["storage"].reset(init_storage=init[ai])
        env.load_component_state()
        if every and env.pf_solver.od_table:
            _unfit(env.pf_solver, every)
    g = torch.Generator(DEV).manual_seed(3)
    listed = 0
    for t in range(steps):
        a = torch.rand((5, n, 8), dtype=torch.float64, device=DEV, generator=g) * 2.2 - 1.1
        outs = []
        for env in envs:
            o, r, d, m = env.step(a)
            outs.append([env.packed_obs().clone(), torch.stack([r[x.name] for x in env.agents]).clone(),
                         m["voltage_violation"].clone(), env.pf_solver.get_bus_voltage_by_name("675c").clone(),
                         env.pf_solver.iterations.clone(), env._fused["agent_power"].clone()])
        F = envs[0]._fused
        listed += int(F["od_count"][F["bufs"].od_parity & 1])
        for i, (x, y) in enumerate(zip(outs[0], outs[1])):
            assert torch.equal(x, y), "split vs two-kernel: step %d output %d" % (t, i)
        if every == 1:
            for i, (x, y) in enumerate(zip(outs[0], outs[2])):
                assert torch.equal(x, y), "all unfit vs no table: step %d output %d" % (t, i)
    if every == 1:
        assert listed == n * steps, listed
    elif every == 3:
        assert 0 < listed < n * steps
    assert (envs[0].pf_solver.iterations > 0).all()


def test_od_row_records_equal_the_currents_rows():
    """Row records (pgw_pf_od.resp_q): the heterogeneous scenario's fused step
    (extrema-only solve, blocks the table serves read the quartic rows alone)
    against the same step with the rows formed from the currents
    (od_row_records=False): the same iteration counts, the voltage extrema and
    the PV farm's min_voltage observation within 1e-12 rel, the rewards within
    1e-9 rel, over 30 steps at 8 192 envs; and the generic path equals the
    fused one bit for bit with the row records on, as does the fused step
    without the per-record candidate slots (od_record_rows=False: every listed
    row of a served env evaluated)."""
    from powergridworld_amd.multiagent_env import MultiAgentEnv
    from powergridworld_amd.scenarios.heterogeneous import make_env_config
    n = 8192
    envs = [MultiAgentEnv(**make_env_config(), num_envs=n, device=DEV, fused=f)
            for f in (True, True, False, True)]
    envs[1].pf_solver.od_row_records = False
    envs[1].pf_solver._tables_cache.clear()
    envs[3].pf_solver.od_record_rows = False
    envs[3].pf_solver._tables_cache.clear()
    envs[3].pf_solver._od_qinfo.clear()
    for env in envs:
        # the same vehicles and initial SoCs in every env (unseeded, each
        # randomize=True component draws its own: the bus loads would differ)
        for k, ag in enumerate(env.agents):
            for c in (ag.envs if hasattr(ag, "envs") else [ag]):
                if hasattr(c, "seed"):
                    c.seed(70 + k)
        env.reset()
    assert envs[0].pf_solver._od_qinfo and any(v is not None for v in envs[0].pf_solver._od_qinfo.values())
    st0 = envs[0].pf_solver.od_resp_stats
    assert 0 < st0["record_rows_candidates"] < st0["record_rows_listed"], st0
    rng = np.random.default_rng(31)
    for t in range(30):
        a = torch.tensor(rng.uniform(-1.1, 1.1, (n, 10)), device=DEV)
        act = {"building": {"building": a[:, :6], "pv": a[:, 6:7], "storage": a[:, 7:8]},
               "pv": a[:, 8:9], "ev-charging": a[:, 9:10]}
        outs = []
        for env in envs:
            o, r, d, m = env.step(act)
            vmin, vmax = env.pf_solver.voltage_extrema()
            outs.append((vmin.clone(), vmax.clone(), env.pf_solver.iterations.clone(),
                         torch.stack([r[k] for k in sorted(r)]).clone()))
        (a0, b0, i0, r0), (a1, b1, i1, r1), (a2, b2, i2, r2), (a3, b3, i3, r3) = outs
        assert torch.equal(i0, i1) and torch.equal(i0, i2) and torch.equal(i0, i3)
        assert torch.equal(a0, a3) and torch.equal(b0, b3) and torch.equal(r0, r3)
        assert ((a0 - a1).abs() / a1).max().item() < 1e-12 and ((b0 - b1).abs() / b1).max().item() < 1e-12
        assert ((r0 - r1).abs() / (1e-3 + r1.abs())).max().item() < 1e-9
        for nm, x, y in (("vmin", a0, a2), ("vmax", b0, b2), ("reward", r0, r2)):
            bad = (x != y).nonzero()
            assert not len(bad), "step %d %s: %d envs differ, e.g. %s: %r vs %r" % (
                t, nm, len(bad), bad[:3].tolist(), x[tuple(bad[0])].item(), y[tuple(bad[0])].item())


# ------------------------------------------------------------------ fp32 storage (pgw_pf_solve_f32)
@pytest.mark.parametrize("conv", ["opendss", "opendss_no_table", "exact"])
def test_pf_solve_f32_equals_fp64_solve(conv):
    """pgw_pf_solve_f32 (SURVEY 8(b)'s fp32 entry): float controllable powers
    in, float node voltages out, the fp64 solve in between -- every output the
    fp64 entry's value on the same (widened) inputs rounded once, every
    iteration count equal, at 4 096 envs over four hours, under the OpenDSS
    rule (with and without the response table) and the exact fixed point."""
    from powergridworld_amd import _lib
    K = 4096
    kw = dict(convergence="exact") if conv == "exact" else {}
    if conv == "opendss_no_table":
        kw["od_table"] = False
    from powergridworld_amd.distribution_system.opendss import OpenDSSSolver
    s = OpenDSSSolver(IEEE13, SHAPE, device=DEV, system_load_rescale_factor=1.2, num_envs=K,
                      **dict({"convergence": "opendss"}, **kw))
    lib = _lib.lib()
    st = _lib.stream_ptr(torch.device(DEV))
    for t, (p, q) in zip(TIMES, _loads(K, 7)):
        s.calculate_power_flow({"675c": torch.tensor(p, device=DEV)}, None, current_time=t)   # tables built
        prm, tb = s.step_params(t), s.solve_tables(t, True)
        n_out = prm.n_out
        p32 = torch.tensor(p, dtype=torch.float32, device=DEV)[None].contiguous()
        p64 = p32.double()
        v64 = torch.empty((n_out, K), dtype=torch.float64, device=DEV)
        v32 = torch.empty((n_out, K), dtype=torch.float32, device=DEV)
        i64 = torch.empty(K, dtype=torch.int32, device=DEV)
        i32 = torch.empty(K, dtype=torch.int32, device=DEV)
        _lib.check(lib.pgw_pf_solve(prm, tb, K, _lib.dptr(p64), None, _lib.dptr(v64), _lib.dptr(i64), st))
        _lib.check(lib.pgw_pf_solve_f32(prm, tb, K, _lib.dptr(p32), None, _lib.dptr(v32), _lib.dptr(i32), st))
        torch.cuda.synchronize()
        assert torch.equal(i64, i32), t
        assert torch.equal(v64.float(), v32), t
        assert (i64 != 0).all() and torch.isfinite(v64).all()
