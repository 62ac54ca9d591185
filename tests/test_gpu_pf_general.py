"""The general batched power flow (pgw_pf_solve_general, csrc/pgw_pf_general.hip):
feeders beyond the 16 load-phase elements of the fast kernels, and OpenDSS's
own snap-solve stopping rule (OpenDSSSolver(convergence="opendss")).  Needs an
MI355X.

PF parity is unpinned (no OpenDSS in this image): every result
is checked against the oracle's independent NumPy restatement --
oracle/pf_oracle.py Feeder.solve (the fixed point) and Feeder.snap_opendss
(OpenDSS's stopped iterate: loads' Yeq in Y, direct-solution start, node
magnitude test at 1e-4, min 2 / max 15 iterations) -- and, for the fixed
point, against the nodal equations themselves.
"""
import os

import numpy as np
import pandas as pd
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
HERE = os.path.dirname(os.path.abspath(__file__))
FEEDER48 = os.path.join(HERE, "data", "feeder48.dss")
MODELS = os.path.join(HERE, "data", "models_feeder.dss")
XFMR3 = os.path.join(HERE, "data", "xfmr3_feeder.dss")
REGCTL = os.path.join(HERE, "data", "regctl_feeder.dss")
REGCTL2 = os.path.join(HERE, "data", "regctl2_feeder.dss")
IEEE13 = "ieee_13_dss/IEEE13Nodeckt.dss"
SHAPE = "ieee_13_dss/annual_hourly_load_profile.csv"


def _solver(feeder, **kw):
    """convergence: "exact" unless a test asks for OpenDSS's rule (the solver's default)."""
    from powergridworld_amd.distribution_system.opendss import OpenDSSSolver
    kw.setdefault("convergence", "exact")
    return OpenDSSSolver(feeder, SHAPE, device=DEV, **kw)


def _oracle(feeder_file, rescale):
    from oracle.pf_oracle import BatchedPF
    from powergridworld_amd.distribution_system.feeder import load_feeder_spec
    spec = load_feeder_spec(feeder_file) if os.path.exists(feeder_file) else None
    return BatchedPF(spec=spec, system_load_rescale_factor=rescale)


def _run(solver, oracle, times, ctrl, lo, hi, K, rng, semantics):
    """Solve K envs with random controllable P / Q at each time; return
    (gpu pu [T, K, n], oracle pu, gpu iterations, oracle iterations)."""
    g_v, o_v, g_it, o_it = [], [], [], []
    f = oracle.feeder
    for t in times:
        p = rng.uniform(lo, hi, K)
        q = rng.uniform(-0.3, 0.5, K) * np.abs(p)
        solver.calculate_power_flow({ctrl: torch.tensor(p, device=DEV)}, {ctrl: torch.tensor(q, device=DEV)},
                                    current_time=t)
        torch.cuda.synchronize()
        bv = solver.get_bus_voltages()
        g_v.append(np.stack([bv[nm].cpu().numpy() for nm in f.node_names], 1))
        g_it.append(solver.iterations.cpu().numpy().copy())
        kw, kvar = oracle.loads(t, {ctrl: p}, {ctrl: q}, K=K)
        if semantics == "opendss":
            V, it = f.snap_opendss(kw, kvar, f.base_kw, f.base_kvar)
        elif semantics == "opendss_h1":                     # every solve's own Yeq in Y
            V, it = f.snap_opendss(kw, kvar)
        else:
            V, it = f.solve(kw, kvar, tol=1e-12)
        o_v.append(f.pu(V))
        o_it.append(it)
    return np.array(g_v), np.array(o_v), np.array(g_it), np.array(o_it)


TIMES = [pd.Timestamp("08-12-2021 %02d:10:00" % h) for h in (3, 11, 17, 20)]


def test_general_kernel_exact_ieee13_vs_oracle():
    """The general kernel forced on IEEE-13 (exact fixed point at 1e-10)
    against the oracle's fixed point at 1e-12: every node within 1e-9 rel."""
    s = _solver(IEEE13, system_load_rescale_factor=1.2, num_envs=3000, general=True)
    assert s.general and s.M == 16
    g, o, git, _ = _run(s, _oracle(IEEE13, 1.2), TIMES, "675c", -400.0, 900.0, 3000,
                        np.random.default_rng(1), "exact")
    assert (git > 0).all()
    np.testing.assert_allclose(g, o, rtol=1e-9, atol=0)
    # the general and the fast kernel solve the same equations
    f = _solver(IEEE13, system_load_rescale_factor=1.2, num_envs=3000)
    assert not f.general
    g2, _, _, _ = _run(f, _oracle(IEEE13, 1.2), TIMES, "675c", -400.0, 900.0, 3000,
                       np.random.default_rng(1), "exact")
    np.testing.assert_allclose(g2, g, rtol=1e-9, atol=0)


def test_opendss_semantics_ieee13_vs_oracle():
    """convergence="opendss": the same stopped iterate as the oracle's
    restatement of OpenDSS's snap solve -- the same iteration count for every
    env, every node within 1e-9 rel -- and measurably not the fixed point."""
    K = 4096
    s = _solver(IEEE13, system_load_rescale_factor=1.2, num_envs=K, convergence="opendss", general=True)
    assert s.general and s.tol == 1e-4 and s.max_iter == 15 and s.min_iter == 2
    g, o, git, oit = _run(s, _oracle(IEEE13, 1.2), TIMES, "675c", -400.0, 900.0, K,
                          np.random.default_rng(2), "opendss")
    np.testing.assert_array_equal(git, oit)
    assert set(np.unique(git)) <= set(range(2, 16))
    np.testing.assert_allclose(g, o, rtol=1e-9, atol=0)
    x = _solver(IEEE13, system_load_rescale_factor=1.2, num_envs=K)
    gx, _, _, _ = _run(x, _oracle(IEEE13, 1.2), TIMES, "675c", -400.0, 900.0, K,
                       np.random.default_rng(2), "exact")
    gap = np.abs(g - gx).max()
    assert 1e-7 < gap < 1e-4          # the stopped iterate is within OpenDSS's tolerance, not at the point


def test_opendss_snap_start_previous_vs_oracle():
    """OpenDSSSolver(snap_start="previous"): each env's snap solve starts from
    its previous solution (the other reading of `Solve mode=snap`,
    opendss.py:134) -- against the oracle's snap_opendss chained through
    V_start over six consecutive solves (the first from the direct solution):
    the same iteration count for every env, every node within 1e-9 rel; and
    measurably not the direct-start reading (the default)."""
    K = 2048
    times = [pd.Timestamp("08-12-2021 11:%02d:00" % m) for m in (0, 5, 10)] + \
            [pd.Timestamp("08-12-2021 12:%02d:00" % m) for m in (0, 5, 10)]
    s = _solver(IEEE13, system_load_rescale_factor=1.2, num_envs=K, convergence="opendss", snap_start="previous")
    d = _solver(IEEE13, system_load_rescale_factor=1.2, num_envs=K, convergence="opendss")
    assert s.general and s.warm_start and not s.od_table
    orc = _oracle(IEEE13, 1.2)
    f = orc.feeder
    rng = np.random.default_rng(41)
    V_prev, gaps = None, []
    for i, t in enumerate(times):
        p = rng.uniform(-400.0, 900.0, K)
        q = rng.uniform(-0.3, 0.5, K) * np.abs(p)
        for x in (s, d):
            x.calculate_power_flow({"675c": torch.tensor(p, device=DEV)}, {"675c": torch.tensor(q, device=DEV)},
                                   current_time=t)
        torch.cuda.synchronize()
        bv, bd = s.get_bus_voltages(), d.get_bus_voltages()
        g = np.stack([bv[nm].cpu().numpy() for nm in f.node_names], 1)
        gd = np.stack([bd[nm].cpu().numpy() for nm in f.node_names], 1)
        kw, kvar = orc.loads(t, {"675c": p}, {"675c": q}, K=K)
        V, it = f.snap_opendss(kw, kvar, f.base_kw, f.base_kvar, V_start=V_prev)
        np.testing.assert_array_equal(s.iterations.cpu().numpy(), it)
        np.testing.assert_allclose(g, f.pu(V), rtol=1e-9, atol=0)
        V_prev = V
        gaps.append(np.abs(g - gd).max())
    assert gaps[0] < 1e-10 and max(gaps[1:]) > 1e-7, gaps      # the first solve starts direct in both


@pytest.mark.parametrize("ctrl", ["675c", "671"])
def test_opendss_yprim_step_vs_oracle(ctrl):
    """OpenDSSSolver(yprim="step"): every snap solve's Y holds its own loads'
    Yeq (the hour's base loads and each env's controllable power -- the reading
    in which the Loads.kW / kvar setters re-stamp Yprim, H1) -- against the
    oracle's snap_opendss with yprim_kw=None over four hours: the same
    iteration count for every env, every node within 1e-9 rel.  675c: one
    controllable phase element (a scalar correction per env); 671: three
    (delta) elements, a 3 x 3 correction per env.  And measurably not the
    default reading (yprim="dss_file", H2)."""
    K = 2048
    s = _solver(IEEE13, system_load_rescale_factor=1.2, num_envs=K, convergence="opendss", yprim="step")
    assert s.general and not s.od_table and s.yprim == "step"
    g, o, git, oit = _run(s, _oracle(IEEE13, 1.2), TIMES, ctrl, -400.0, 900.0, K,
                          np.random.default_rng(5), "opendss_h1")
    assert s.params.r_reg == (1 if ctrl == "675c" else 3)
    np.testing.assert_array_equal(git, oit)
    np.testing.assert_allclose(g, o, rtol=1e-9, atol=0)
    d = _solver(IEEE13, system_load_rescale_factor=1.2, num_envs=K, convergence="opendss", general=True)
    gd, _, _, _ = _run(d, _oracle(IEEE13, 1.2), TIMES, ctrl, -400.0, 900.0, K,
                       np.random.default_rng(5), "opendss")
    assert np.abs(g - gd).max() > 1e-7


def test_het_yprim_step_runs_the_generic_path():
    """The heterogeneous scenario with yprim="step": the fused step refuses it
    (its kernels hold the DSS file's Yeq), the generic path runs it -- the PV
    farm's min-voltage observation and the rewards finite, every env's solve
    within OpenDSS's iteration limits."""
    from powergridworld_amd.multiagent_env import MultiAgentEnv
    from powergridworld_amd.scenarios.heterogeneous import make_env_config
    cfg = make_env_config()
    cfg["pf_config"]["config"]["yprim"] = "step"
    env = MultiAgentEnv(**cfg, num_envs=256, device=DEV)
    assert env._ma is None and env.pf_solver.yprim == "step"
    rng = np.random.default_rng(8)
    env.reset()
    for _ in range(12):
        a = torch.tensor(rng.uniform(-1, 1, (256, 10)), device=DEV)
        o, r, d, m = env.step({"building": {"building": a[:, :6], "pv": a[:, 6:7], "storage": a[:, 7:8]},
                               "pv": a[:, 8:9], "ev-charging": a[:, 9:10]})
        it = env.pf_solver.iterations
        assert bool(((it >= 2) & (it <= 15)).all())
        assert all(bool(torch.isfinite(v).all()) for v in r.values())


def test_large_feeder_exact_and_opendss_vs_oracle():
    """A 48-element synthetic feeder (tests/data/feeder48.dss; the fast kernels
    stop at 16): exact fixed point and OpenDSS semantics against the oracle,
    the fixed point also against the nodal equations."""
    from powergridworld_amd.distribution_system.feeder import load_feeder_spec
    from oracle.pf_oracle import Feeder as OracleFeeder
    K = 2048
    o = _oracle(FEEDER48, 1.0)
    assert o.feeder.Cinc.shape[0] == 48
    s = _solver(FEEDER48, num_envs=K)
    assert s.general and s.M == 48
    g, ov, git, _ = _run(s, o, TIMES, "f1", -200.0, 600.0, K, np.random.default_rng(3), "exact")
    assert (git > 0).all()
    np.testing.assert_allclose(g, ov, rtol=1e-8, atol=0)
    # nodal residual of a GPU solution: the voltages the kernel reports are
    # magnitudes, so check the oracle fixed point they match instead, at one env
    f = OracleFeeder(load_feeder_spec(FEEDER48))
    kw, kvar = o.loads(TIMES[1], {"f1": np.array([350.0])}, None, K=1)
    V, _ = f.solve(kw, kvar, tol=1e-13)
    W_ph = kw[:, f.elem_load] * 1000.0 / f.elem_nph
    var_ph = kvar[:, f.elem_load] * 1000.0 / f.elem_nph
    I = f.load_currents((f.Cinc @ V[0])[None], W_ph, var_ph)[0]
    resid = np.abs(f.Y @ V[0] - (f.I_src - f.Cinc.T @ I)).max() / np.abs(f.I_src).max()
    assert resid < 1e-8
    d = _solver(FEEDER48, num_envs=K, convergence="opendss")
    g2, o2, git2, oit2 = _run(d, o, TIMES, "f1", -200.0, 600.0, K, np.random.default_rng(4), "opendss")
    np.testing.assert_array_equal(git2, oit2)
    np.testing.assert_allclose(g2, o2, rtol=1e-9, atol=0)


def test_load_models_and_series_capacitor_vs_oracle():
    """OpenDSS load models 1-8 and a series capacitor (tests/data/models_feeder.dss):
    the general kernel's current laws (fixed point and OpenDSS semantics)
    against the oracle's (Feeder.LAWS), every node within 1e-9 rel, the same
    OpenDSS iteration counts; only the model-1 loads take the loadshape and the
    controllable power.  Parity unpinned (no OpenDSS)."""
    K = 2048
    o = _oracle(MODELS, 1.1)
    s = _solver(MODELS, system_load_rescale_factor=1.1, num_envs=K)
    assert s.general and s.feeder.m == 16 and (s.feeder.elem_model != 1).any()
    g, ov, git, _ = _run(s, o, TIMES, "pq1", -100.0, 400.0, K, np.random.default_rng(7), "exact")
    assert (git > 0).all()
    np.testing.assert_allclose(g, ov, rtol=1e-9, atol=0)
    d = _solver(MODELS, system_load_rescale_factor=1.1, num_envs=K, convergence="opendss")
    g2, o2, git2, oit2 = _run(d, o, TIMES, "pq1", -100.0, 400.0, K, np.random.default_rng(8), "opendss")
    np.testing.assert_array_equal(git2, oit2)
    np.testing.assert_allclose(g2, o2, rtol=1e-9, atol=0)


def test_three_winding_and_centre_tap_transformers_vs_oracle():
    """3-winding and centre-tapped transformers (tests/data/xfmr3_feeder.dss,
    the native N-winding element): the fast kernel, the general kernel and
    OpenDSS semantics against the oracle's independent stamp, every node within
    1e-9 rel.  Parity unpinned (no OpenDSS)."""
    K = 2048
    o = _oracle(XFMR3, 1.0)
    for general in (False, True):
        s = _solver(XFMR3, num_envs=K, general=general)
        assert s.general == general and s.feeder.m == 16
        g, ov, git, _ = _run(s, o, TIMES, "x1", -300.0, 500.0, K, np.random.default_rng(9), "exact")
        assert (git > 0).all()
        np.testing.assert_allclose(g, ov, rtol=1e-9, atol=0)
    d = _solver(XFMR3, num_envs=K, convergence="opendss")
    g2, o2, git2, oit2 = _run(d, o, TIMES, "x1", -300.0, 500.0, K, np.random.default_rng(10), "opendss")
    np.testing.assert_array_equal(git2, oit2)
    np.testing.assert_allclose(g2, o2, rtol=1e-9, atol=0)


@pytest.mark.parametrize("feeder", ["regctl", "regctl2"])
@pytest.mark.parametrize("semantics", ["exact", "opendss"])
def test_regcontrol_vs_oracle(semantics, feeder):
    """RegControl (tests/data/regctl_feeder.dss: three single-phase regulators,
    one with line-drop compensation, and a gang-operated 3-phase one;
    regctl2_feeder.dss: Sample's options -- a remote regulated bus, Vlimit
    over line-drop compensation, inverse time, PTphase=max / min): per-env
    taps through the Woodbury-corrected general kernel and the device control
    pass (pgw_reg_control / pgw_reg_factor) against the oracle's SolveSnap
    restatement that rebuilds and re-inverts Y at every tap set -- the same
    final taps in every env (exactly), every node within 1e-9 rel, over two
    consecutive steps (taps persist) from random per-env starting taps.
    Parity unpinned (no OpenDSS)."""
    K = 192
    path = {"regctl": REGCTL, "regctl2": REGCTL2}[feeder]
    o = _oracle(path, 1.0)
    s = _solver(path, num_envs=K, convergence=semantics)
    f = o.feeder
    reg = s.regulators
    nc = len(reg["ctrls"])
    assert s.general and reg is not None and nc == {"regctl": 4, "regctl2": 5}[feeder]
    rng = np.random.default_rng(11)
    taps = reg["taps0"][None, :] + 0.00625 * rng.integers(-6, 7, size=(K, nc))
    s.set_regulator_taps(torch.tensor(taps.T.copy(), device=DEV))
    moved = 0
    for t in TIMES[1:3]:
        p = rng.uniform(-300.0, 900.0, K)
        q = rng.uniform(-0.3, 0.5, K) * np.abs(p)
        s.calculate_power_flow({"f1": torch.tensor(p, device=DEV)}, {"f1": torch.tensor(q, device=DEV)},
                               current_time=t)
        torch.cuda.synchronize()
        bv = s.get_bus_voltages()
        g = np.stack([bv[nm].cpu().numpy() for nm in f.node_names], 1)
        gt = s.reg_taps.cpu().numpy().T
        kw, kvar = o.loads(t, {"f1": p}, {"f1": q}, K=K)
        if semantics == "opendss":
            V, it, tp, cp = f.solve_regulated(kw, kvar, taps, "opendss", f.base_kw, f.base_kvar)
        else:
            V, it, tp, cp = f.solve_regulated(kw, kvar, taps)
        np.testing.assert_array_equal(gt, tp)
        np.testing.assert_allclose(g, f.pu(V), rtol=1e-9, atol=0)
        if semantics == "opendss":
            np.testing.assert_array_equal(s.iterations.cpu().numpy(), it)
        assert s.control_iterations == cp.max()
        moved += int((tp != taps).any(1).sum())
        taps = tp
    assert moved > K // 4


def test_general_kernel_extrema_and_output_subset():
    """Output-row subsets and the min / max epilogue of the general kernel."""
    K = 1000
    s = _solver(FEEDER48, num_envs=K, convergence="opendss")
    full = _solver(FEEDER48, num_envs=K, convergence="opendss")
    names = s.feeder.node_names
    s.set_output_nodes([names[5], names[40], names[2]])
    rng = np.random.default_rng(5)
    p = torch.tensor(rng.uniform(-100, 500, K), device=DEV)
    for solver in (s, full):
        solver.calculate_power_flow({"f1": p}, None, current_time=TIMES[2])
    torch.cuda.synchronize()
    fb = full.get_bus_voltages()
    for nm in (names[5], names[40], names[2]):
        assert torch.equal(s.get_bus_voltages()[nm], fb[nm])
    allv = torch.stack([fb[nm] for nm in names])
    mn, mx = full.voltage_extrema()
    assert torch.equal(mn, allv.min(0).values) and torch.equal(mx, allv.max(0).values)


def test_general_kernel_multi_bus_warm_start():
    """Several controllable loads on the large feeder, exact mode, warm start
    from each env's previous solution: the same fixed point as a cold start."""
    K = 512
    cold = _solver(FEEDER48, num_envs=K)
    warm = _solver(FEEDER48, num_envs=K, warm_start=True)
    rng = np.random.default_rng(6)
    for t in TIMES:
        p = {nm: torch.tensor(rng.uniform(-50, 300, K), device=DEV) for nm in ("w3", "s7", "f1", "d10")}
        for sv in (cold, warm):
            sv.calculate_power_flow(p, None, current_time=t)
        torch.cuda.synchronize()
        a = torch.stack(list(cold.get_bus_voltages().values()))
        b = torch.stack(list(warm.get_bus_voltages().values()))
        torch.testing.assert_close(a, b, rtol=1e-9, atol=0)


def _c4_pair(n, convergence):
    """(fused, generic) C4 envs on the GENERAL power flow (the fast kernels'
    OpenDSS rule: tests/test_gpu_pf_od.py)."""
    from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config
    envs = [CoordinatedMultiBuildingControlEnv(**make_c4_config(pf_convergence=convergence, pf_general=True),
                                               num_envs=n, device=DEV, fused=f) for f in (True, False)]
    return envs


def test_c4_opendss_fused_equals_generic_and_oracle():
    """C4 with convergence="opendss": the fused step (pgw_coord_step_general:
    agents kernel + general PF with the coordinated prologue / epilogue) is
    bit-identical to the generic per-component path, and both match the NumPy
    C4 oracle run with OpenDSS's snap semantics."""
    from oracle.ma_oracle import CoordinatedOracle
    from oracle.pf_oracle import BatchedPF
    n = 256
    fused, generic = _c4_pair(n, "opendss")
    assert fused._fused is not None and fused._fused["kernel"] == "pgw_coord_step_general"
    assert generic._fused is None and generic.pf_solver.convergence == "opendss"
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
        np.testing.assert_allclose(mf["voltage_violation"].cpu().numpy(), o_vv, rtol=1e-8, atol=1e-11)
        np.testing.assert_array_equal(fused.pf_solver.iterations.cpu().numpy(), ora.pf.last_iters)
    # every other node on demand: the same solve as the generic path's
    v_f, v_g = fused.voltages, generic.voltages
    for nm in ("632.1", "671.2", "652.1", "675.3"):
        assert torch.equal(v_f[nm], v_g[nm])


def test_het_opendss_fused_equals_generic():
    """The heterogeneous scenario with convergence="opendss": pgw_ma_step's
    agents + the OpenDSS-rule PF (fast or general kernel; extrema epilogue for
    the PV farm's min_voltage) bit-identical to the generic path over a stretch
    of the episode."""
    from powergridworld_amd.multiagent_env import MultiAgentEnv
    from powergridworld_amd.scenarios.heterogeneous import make_env_config
    n = 512
    envs = [MultiAgentEnv(**make_env_config(pf_convergence="opendss"), num_envs=n, device=DEV, fused=f)
            for f in ("auto", False)]
    assert envs[0]._ma is not None and envs[1]._ma is None
    # one controllable bus: the fast OpenDSS-rule kernel (k_pf_solve_od); more: the general one
    assert (envs[0]._ma["general"] is None) == envs[0].pf_solver._od_fast
    rng = np.random.default_rng(12)
    for e in envs:
        for k, a in enumerate(e.agents):
            for c in (a.envs if hasattr(a, "envs") else [a]):
                if hasattr(c, "seed"):
                    c.seed(50 + k)
        e.reset()
    for t in range(60):
        act = {"building": {"building": torch.tensor(rng.uniform(-1, 1, (n, 6)), device=DEV),
                            "pv": torch.tensor(rng.uniform(-1, 1, (n, 1)), device=DEV),
                            "storage": torch.tensor(rng.uniform(-1, 1, (n, 1)), device=DEV)},
               "pv": torch.tensor(rng.uniform(-1, 1, (n, 1)), device=DEV),
               "ev-charging": torch.tensor(rng.uniform(-1, 1, (n, 1)), device=DEV)}
        res = [e.step(act) for e in envs]
        torch.cuda.synchronize()
        (o0, r0, _, _), (o1, r1, _, _) = res
        for name in r0:
            assert torch.equal(r0[name], r1[name]), (t, name)
        assert torch.equal(o0["pv"], o1["pv"])
        assert torch.equal(envs[0].pf_solver.iterations, envs[1].pf_solver.iterations)


def test_het_extrema_rows_mask_changes_nothing():
    """pgw_pf_od.resp_rows (OpenDSSSolver._od_row_mask): the heterogeneous
    scenario's extrema evaluated on the rows the host proved can hold a served
    env's minimum or maximum |V| are bit-identical to every row's -- the
    rewards, the PV farm's min-voltage observation, the iteration counts and
    both extrema, over 60 steps at 8 192 envs -- and the masks are non-trivial
    (fewer rows than the outputs)."""
    from powergridworld_amd.multiagent_env import MultiAgentEnv
    from powergridworld_amd.scenarios.heterogeneous import make_env_config
    n = 8192
    envs = [MultiAgentEnv(**make_env_config(pf_convergence="opendss"), num_envs=n, device=DEV) for _ in range(2)]
    envs[1].pf_solver.od_row_masks = False
    rng = np.random.default_rng(13)
    for e in envs:
        for k, a in enumerate(e.agents):
            for c in (a.envs if hasattr(a, "envs") else [a]):
                if hasattr(c, "seed"):
                    c.seed(60 + k)
        e.reset()
    s0 = envs[0].pf_solver
    masks = [m for (idx, cfg), m in s0._od_rowmask.items()]
    n_out = len(s0.output_names)
    assert masks and all(0 < bin(m).count("1") < n_out - 1 for m in masks), (n_out, [bin(m).count("1") for m in masks])
    for t in range(60):
        act = {"building": {"building": torch.tensor(rng.uniform(-1, 1, (n, 6)), device=DEV),
                            "pv": torch.tensor(rng.uniform(-1, 1, (n, 1)), device=DEV),
                            "storage": torch.tensor(rng.uniform(-1, 1, (n, 1)), device=DEV)},
               "pv": torch.tensor(rng.uniform(-1, 1, (n, 1)), device=DEV),
               "ev-charging": torch.tensor(rng.uniform(-1, 1, (n, 1)), device=DEV)}
        res = [e.step(act) for e in envs]
        torch.cuda.synchronize()
        (o0, r0, _, _), (o1, r1, _, _) = res
        for name in r0:
            assert torch.equal(r0[name], r1[name]), (t, name)
        assert torch.equal(o0["pv"], o1["pv"]), t
        assert torch.equal(envs[0].pf_solver.iterations, envs[1].pf_solver.iterations)
        for x, y in zip(envs[0].pf_solver.voltage_extrema(), envs[1].pf_solver.voltage_extrema()):
            assert torch.equal(x, y), t


def test_regcontrol_multiagent_generic_path():
    """A MultiAgentEnv on the RegControl feeder (PV farm, EV station and battery
    agents on its loads f1 / a1 / f2): the fused paths step aside (the control
    loop lives in calculate_power_flow), the generic path's node voltages and
    the regulators' taps follow the oracle's SolveSnap restatement driven by the
    agents' own real powers, step after step (taps carried).  Parity unpinned."""
    from powergridworld_amd.agents import EnergyStorageEnv
    from powergridworld_amd.agents.vehicles import EVChargingEnv
    from powergridworld_amd.distribution_system.opendss import OpenDSSSolver
    from powergridworld_amd.multiagent_env import MultiAgentEnv
    from powergridworld_amd.scenarios.heterogeneous import ThisPVEnv
    K = 128
    cfg = {"common_config": {"start_time": "08-12-2020 06:00:00", "end_time": "08-13-2020 00:00:00",
                             "control_timedelta": pd.Timedelta(300, "s")},
           "pf_config": {"cls": OpenDSSSolver,
                         "config": {"feeder_file": REGCTL, "loadshape_file": SHAPE,
                                    "system_load_rescale_factor": 1.0, "convergence": "exact"}},
           "agents": [
               {"name": "pv", "bus": "f1", "cls": ThisPVEnv,
                "config": {"profile_csv": "off-peak.csv", "scaling_factor": 400., "grid_aware": True}},
               {"name": "ev", "bus": "a1", "cls": EVChargingEnv,
                "config": {"num_vehicles": 25, "minutes_per_step": 5, "max_charge_rate_kw": 7.,
                           "peak_threshold": 200., "vehicle_multiplier": 20.}},
               {"name": "storage", "bus": "f2", "cls": EnergyStorageEnv,
                "config": {"max_power": 150., "storage_range": (3., 250.)}}]}
    env = MultiAgentEnv(**cfg, num_envs=K, device=DEV)
    assert env._fused is None and env._ma is None
    o = _oracle(REGCTL, 1.0)
    f = o.feeder
    env.reset()
    s = env.pf_solver
    taps = s.reg_taps.cpu().numpy().T.copy()
    rng = np.random.default_rng(21)
    moved = 0
    for t in range(12):
        a = {"pv": T(rng.uniform(-1, 1, (K, 1))), "ev": T(rng.uniform(-1, 1, (K, 1))),
             "storage": T(rng.uniform(-1, 1, (K, 1)))}
        env.step(a)
        torch.cuda.synchronize()
        p = {bus: env.agent_dict[nm].real_power.cpu().numpy() for nm, bus in (("pv", "f1"), ("ev", "a1"),
                                                                              ("storage", "f2"))}
        kw, kvar = o.loads(env.time, p, None, K=K)
        V, it, tp, cp = f.solve_regulated(kw, kvar, taps)
        np.testing.assert_array_equal(s.reg_taps.cpu().numpy().T, tp)
        bv = s.get_bus_voltages()
        g = np.stack([bv[nm].cpu().numpy() for nm in f.node_names], 1)
        np.testing.assert_allclose(g, f.pu(V), rtol=1e-9, atol=0)
        moved += int((tp != taps).any(1).sum())
        taps = tp
    assert moved > 0


def T(x):
    return torch.tensor(np.asarray(x, dtype=np.float64), device=DEV)
