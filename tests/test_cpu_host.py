"""CPU-only checks: the C ABI library loads and exports every symbol pgw.h
declares, struct layouts agree, the native feeder build agrees with the
oracle, the DSS parser, the PF formulation satisfies the nodal equations,
and host-side data/config logic."""
import os
import re

import numpy as np
import pytest

from tests.conftest import REPO


def test_library_exports_every_header_symbol():
    from powergridworld_amd import _lib
    h = _lib.lib()     # also verifies ABI version and every struct size
    header = open(os.path.join(REPO, "include", "pgw.h")).read()
    declared = set(re.findall(r"\b(pgw_[a-z0-9_]+)\s*\(", header))
    assert declared, "no declarations parsed"
    for name in declared:
        assert hasattr(h, name), name
    assert declared <= set(_lib.EXPORTED), declared - set(_lib.EXPORTED)


def test_feeder_native_build_matches_oracle():
    from oracle.pf_oracle import Feeder as OracleFeeder, load_ieee13
    from powergridworld_amd.distribution_system.feeder import Feeder, load_feeder_spec
    f = Feeder(load_feeder_spec("ieee_13_dss/IEEE13Nodeckt.dss"))
    o = OracleFeeder(load_ieee13())
    assert f.node_names == o.node_names and f.n == 38
    # Y is ill-conditioned (~1e7); both sides invert it in extended precision
    np.testing.assert_allclose(f.Y, o.Y, rtol=1e-12, atol=1e-9)
    assert np.abs(f.Z - o.Z).max() / np.abs(o.Z).max() < 1e-10
    np.testing.assert_allclose(f.kv_ln, o.kv_ln, rtol=1e-15)
    M, W, U0, G, V0 = f.reduce([f.node_index["675.3"], f.node_index["634.1"]])
    assert M == 14 and f.m == 14
    assert np.abs(W[:f.m, :f.m] - o.W).max() / np.abs(o.W).max() < 1e-10
    assert np.abs(U0[:f.m] - o.U0).max() / np.abs(o.U0).max() < 1e-10


def test_dss_parser_ieee13():
    from powergridworld_amd.distribution_system.dss import parse_matrix, parse_number
    from powergridworld_amd.distribution_system.feeder import load_feeder_spec
    assert parse_number("(8 1000 /)") == pytest.approx(0.008)
    assert parse_number("(.5 1000 /)") == pytest.approx(0.0005)
    m = parse_matrix("[0.791721  |0.318476  0.781649  |0.28345  0.318476  0.791721  ]")
    assert m[0][2] == m[2][0] == 0.28345
    spec = load_feeder_spec("ieee_13_dss/IEEE13Nodeckt.dss")
    assert [ld["name"] for ld in spec["loads"]][7] == "675c"
    assert spec["source"]["pu"] == 1.0001 and spec["source"]["angle"] == 30
    assert spec["transformers"][0]["xhl"] == pytest.approx(0.008)
    assert spec["voltagebases"] == [115.0, 4.16, 0.48]
    sw = [l for l in spec["lines"] if l["switch"]][0]
    assert sw["length"] == 0.001 and sw["sequence"]["r1"] == 1e-4


def test_pf_fixed_point_solves_nodal_equations():
    """Physical residual: the converged oracle voltages satisfy Y V = I_src + I_loads(V)
    and the power drawn by each element equals its specified S (inside the PQ band)."""
    from oracle.pf_oracle import BatchedPF
    pf = BatchedPF(system_load_rescale_factor=0.7)
    f = pf.feeder
    kw, kvar = pf.base_loads("2021-01-01 05:00")
    V, it = f.solve(kw[None], kvar[None], tol=1e-13)
    W_ph = kw[f.elem_load] * 1000.0 / f.elem_nph
    var_ph = kvar[f.elem_load] * 1000.0 / f.elem_nph
    U = f.Cinc @ V[0]
    I = f.load_currents(U[None], W_ph[None], var_ph[None])[0]
    inj = f.I_src - f.Cinc.T @ I
    resid = np.abs(f.Y @ V[0] - inj).max() / np.abs(f.I_src).max()
    assert resid < 1e-8
    S = U * np.conj(I)
    pu = np.abs(U) / f.elem_vbase
    band = (pu > 0.95) & (pu <= 1.05)
    np.testing.assert_allclose(S.real[band], W_ph[band], rtol=1e-9, atol=1e-6)
    np.testing.assert_allclose(S.imag[band], var_ph[band], rtol=1e-9, atol=1e-6)


FEEDER48 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "feeder48.dss")
REGCAP = os.path.join(REPO, "tests", "data", "regcap_feeder.dss")


def test_dss_regulators_capacitors_model2_loads():
    """The DSS subset beyond IEEE-13 (tests/data/regcap_feeder.dss): 1-phase
    regulators in array form with fixed taps set by property assignment,
    RegControl off, capacitors, model-2 loads.  Parity unpinned (no OpenDSS):
    the native build is checked against the oracle's independent NumPy one and
    the solve against the nodal equations, shunts included."""
    from oracle.pf_oracle import Feeder as OracleFeeder
    from powergridworld_amd.distribution_system.feeder import Feeder, load_feeder_spec
    spec = load_feeder_spec(REGCAP)
    regs = {t["name"]: t for t in spec["transformers"]}
    assert [w["tap"] for w in regs["reg3"]["windings"]] == [1.0, 1.06875]
    assert regs["reg1"]["phases"] == 1 and regs["reg1"]["windings"][1]["bus"] == "RG60.1"
    assert regs["reg1"]["windings"][0]["pct_r"] == pytest.approx(0.005)
    assert spec["controlmode"] == "off" and len(spec["regcontrols"]) == 1
    assert [c["kvar"] for c in spec["capacitors"]] == [600.0, 100.0]
    f, o = Feeder(spec), OracleFeeder(spec)
    assert f.node_names == o.node_names
    assert f.m == 5                      # model-1 phase elements: delta 3 + 2 single-phase
    assert np.abs(f.Y - o.Y).max() / np.abs(o.Y).max() < 1e-12
    assert np.abs(f.Z - o.Z).max() / np.abs(o.Z).max() < 1e-10
    M, W, U0, G, V0 = f.reduce([f.node_index["b4.3"]])
    assert np.abs(W[:f.m, :f.m] - o.W).max() / np.abs(o.W).max() < 1e-10
    # the taps set the no-load ratio of each regulator
    i = f.node_index
    for ph, tap in ((1, 1.0625), (2, 1.05), (3, 1.06875)):
        r = abs(f.V0[i["rg60.%d" % ph]]) / abs(f.V0[i["650.%d" % ph]])
        assert r == pytest.approx(tap, rel=1e-3)     # (line charging and capacitors load it slightly)
    # nodal residual of a converged solve, with the shunts in Y
    kw = np.array([ld["kw"] for ld in spec["loads"]], float)
    kvar = np.array([ld["kvar"] for ld in spec["loads"]], float)
    V, it = o.solve(kw[None], kvar[None], tol=1e-13)
    W_ph = kw[o.elem_load] * 1000.0 / o.elem_nph
    var_ph = kvar[o.elem_load] * 1000.0 / o.elem_nph
    U = o.Cinc @ V[0]
    I = o.load_currents(U[None], W_ph[None], var_ph[None])[0]
    resid = np.abs(o.Y @ V[0] - (o.I_src - o.Cinc.T @ I)).max() / np.abs(o.I_src).max()
    assert resid < 1e-8


def test_dss_unsupported_control_and_models_refused(tmp_path):
    from powergridworld_amd.distribution_system.feeder import Feeder, load_feeder_spec
    text = open(REGCAP).read()
    p = tmp_path / "ctl.dss"
    p.write_text(text.replace("Set Controlmode=OFF", ""))
    assert len(Feeder(load_feeder_spec(str(p))).regulators()["ctrls"]) == 1     # STATIC: simulated
    assert Feeder(load_feeder_spec(REGCAP)).regulators() is None                  # OFF: fixed taps
    p.write_text(text.replace("Set Controlmode=OFF", "").replace("R=3 X=9", "R=3 X=9 reversible=yes"))
    with pytest.raises(NotImplementedError, match="reversible"):
        Feeder(load_feeder_spec(str(p))).regulators()
    p.write_text(text.replace("Set Controlmode=OFF", "Set Controlmode=TIME"))
    with pytest.raises(NotImplementedError, match="Controlmode"):
        Feeder(load_feeder_spec(str(p)))
    p = tmp_path / "m9.dss"
    p.write_text(text.replace("Model=2 kV=2.4", "Model=9 kV=2.4"))
    with pytest.raises(NotImplementedError, match="model 9"):
        Feeder(load_feeder_spec(str(p)))


def test_feeder48_native_build_and_opendss_model():
    """The 48-element synthetic feeder (tests/data/feeder48.dss, beyond the fast
    kernels' 16): native Y / Z equal the oracle's NumPy build; with the loads'
    nominal admittances stamped (OpenDSS's iteration matrix, load_yprim) Y
    grows by exactly C^T diag(Yeq) C, and the oracle's OpenDSS-semantics solve
    stops within OpenDSS's tolerance of the fixed point."""
    from oracle.pf_oracle import Feeder as OracleFeeder
    from powergridworld_amd.distribution_system.feeder import Feeder, load_feeder_spec
    spec = load_feeder_spec(FEEDER48)
    f, o = Feeder(spec), OracleFeeder(spec)
    assert f.m == 48 and f.node_names == o.node_names
    assert np.abs(f.Y - o.Y).max() / np.abs(o.Y).max() < 1e-12
    assert np.abs(f.Z - o.Z).max() / np.abs(o.Z).max() < 1e-9
    fy = Feeder(spec, load_yprim=True)
    S = (f.base_kw[f.elem_load] - 1j * f.base_kvar[f.elem_load]) * 1000.0 / f.elem_nph
    C = o.Cinc
    np.testing.assert_allclose(fy.Y, f.Y + C.T @ np.diag(S / f.elem_vbase ** 2) @ C, rtol=0,
                               atol=1e-12 * np.abs(f.Y).max())
    kw = np.array([ld["kw"] for ld in spec["loads"]], float)[None]
    kvar = np.array([ld["kvar"] for ld in spec["loads"]], float)[None]
    V, _ = o.solve(1.2 * kw, 1.2 * kvar, tol=1e-12)
    Vd, it = o.snap_opendss(1.2 * kw, 1.2 * kvar, o.base_kw, o.base_kvar)
    assert 2 <= it[0] <= 15
    assert np.abs(o.pu(Vd) - o.pu(V)).max() < 1e-4


def test_dss_edits_of_unsimulated_classes_refused(tmp_path):
    """An Edit / Class.Name.Prop= of a capacitor or line would otherwise leave the
    original element in Y (a wrong network without an error); edits of meters
    and shapes cannot change the network and are ignored.  Extra key=value
    pairs of a property assignment are normalised like New's."""
    from powergridworld_amd.distribution_system.dss import parse_dss
    text = open(REGCAP).read()
    for extra in ("Capacitor.C1.States=[0]", "Edit Capacitor.C1 kvar=300", "Edit Line.650632 enabled=no"):
        p = tmp_path / "e.dss"
        p.write_text(text + "\n" + extra + "\n")
        with pytest.raises(NotImplementedError, match="not supported"):
            parse_dss(str(p))
    p = tmp_path / "ok.dss"
    p.write_text(text + "\nEdit EnergyMeter.m1 element=Line.650632\n"
                 "Transformer.Reg1.Taps=[1.0 1.05] XHL=0.02\n")
    spec = parse_dss(str(p))
    reg1 = {t["name"]: t for t in spec["transformers"]}["reg1"]
    assert [w["tap"] for w in reg1["windings"]] == [1.0, 1.05]
    assert reg1["xhl"] == pytest.approx(0.02)


def test_product_synthetic_exogenous_matches_fixture(exo_frame):
    from powergridworld_amd.agents.buildings import synthetic_exogenous_data
    df = synthetic_exogenous_data()
    assert list(df.columns) == list(exo_frame.columns)
    assert (df.index == exo_frame.index).all()
    np.testing.assert_array_equal(df.values, exo_frame.values)


def test_bus_name_mapping():
    from powergridworld_amd.distribution_system.opendss import bus_name_to_nodes
    assert bus_name_to_nodes("675c") == ["675.3"]
    assert bus_name_to_nodes("634a") == ["634.1"]
    assert bus_name_to_nodes("675") == ["675.1", "675.2", "675.3"]
    # the reference replaces EVERY occurrence of the last char (opendss.py:180)
    assert bus_name_to_nodes("cac") == [".3a.3"]


def test_data_assets():
    from powergridworld_amd.agents.pv import load_profile
    d = load_profile("pv_profile.csv")
    assert d.shape == (287,) and d.max() == 1.0
    assert load_profile("off-peak.csv").shape == (288,)
    ls = np.load(os.path.join(REPO, "powergridworld_amd", "data", "loadshape_8760.npy"))
    assert ls.shape == (8760,)


def test_exact_division(tmp_path):
    """exact_div (pgw_common.h): x * RN(1/d) plus two fma residual corrections
    equals the IEEE quotient bit for bit -- random (x, d) over wide exponent
    ranges, random mantissas, and the C4 divisors (obs ranges, SoC range,
    storage efficiency and step length, the 12 of the building reward)."""
    import subprocess
    exe = str(tmp_path / "div_exact")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe,
                    os.path.join(REPO, "tests", "c", "div_exact.c"), "-lm"], check=True)
    divisors = ["6", "20", "50", "10", "2", "1", "47", "0.9", "0.0833333333333333", "12"]
    r = subprocess.run([exe, "2000000"] + divisors, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "mismatches: 0" in r.stdout


def test_env_tensor_and_action_normalisation():
    """as_env_tensor / as_action (the host side of every step): an [N] fp64
    vector on the device passes through as the same object (the per-step fast
    path), other shapes and dtypes are converted or broadcast, and a shape that
    fits neither raises ValueError as the reference's numpy code would fail."""
    import torch
    from powergridworld_amd.base import as_action, as_env_tensor
    dev = torch.device("cpu")
    v = torch.arange(4, dtype=torch.float64)
    assert as_env_tensor(v, 4, dev) is v
    col = v.reshape(4, 1)
    assert torch.equal(as_env_tensor(col, 4, dev), v)
    assert torch.equal(as_env_tensor(2.5, 4, dev), torch.full((4,), 2.5, dtype=torch.float64))
    assert as_env_tensor(v.float(), 4, dev).dtype == torch.float64
    strided = torch.arange(8, dtype=torch.float64)[::2]
    got = as_env_tensor(strided, 4, dev)
    assert got.is_contiguous() and torch.equal(got, strided)
    with pytest.raises(ValueError):
        as_env_tensor(torch.zeros(3, dtype=torch.float64), 4, dev)
    a = torch.zeros((4, 2), dtype=torch.float64)
    assert as_action(a, 4, 2, dev) is a
    assert tuple(as_action([0.5, -0.5], 4, 2, dev).shape) == (4, 2)       # one action for all envs
    assert tuple(as_action(v, 4, 1, dev).shape) == (4, 1)
    with pytest.raises(ValueError):
        as_action(torch.zeros((3, 2)), 4, 2, dev)


def test_ma_step_argument_checks():
    """pgw_ma_step validates its layout before any HIP call (no GPU needed):
    agents must cover the slots in order, every slot appear once in the waves,
    a building / EV slot have a wave of its own, one building / storage / EV in
    all, and the PF's controllable slots match the bus count."""
    import ctypes as C
    from powergridworld_amd import _lib
    lib = _lib.lib()

    def args(kinds, waves, agents):
        a = _lib.MAStepArgs()
        a.n_comp = len(kinds)
        dummy = 256          # never dereferenced: the checks fail (or pass) first
        n_pv = 0
        for c, k in enumerate(kinds):
            a.comp[c].kind = k
            if k == 1:
                a.slot_pv2[c], n_pv = n_pv, n_pv + 1
            a.comp[c].action = _lib.Mat(dummy, 1, 1)
            a.comp[c].obs = _lib.Mat(dummy, 1, 1)
            a.comp[c].real_power = dummy
        a.bld_x = a.bld_reward_state = a.bat_soc = dummy
        a.ev_endp = a.ev_req = a.ev_charging = a.ev_reward = dummy
        a.n_waves = len(waves)
        i = 0
        for w, cs in enumerate(waves):
            a.wave_first[w], a.wave_count[w] = i, len(cs)
            for c in cs:
                a.wave_slot[i] = c
                i += 1
        a.n_agents = len(agents)
        s = 0
        for g, cnt in enumerate(agents):
            a.agent_first[g], a.agent_count[g], a.agent_bus[g] = s, cnt, -1
            a.agent_sum[g] = int(cnt > 1)
            a.agent_real_power[g] = a.agent_reward[g] = dummy
            for c in range(s, s + cnt):
                a.slot_agent[c] = g
            s += cnt
        return a

    def rc(a):
        r = lib.pgw_ma_step(C.byref(a), None, None, 0, None, None, None)   # n = 0: checks only
        return r, lib.pgw_last_error().decode()

    B, PV, ST, EV = 0, 1, 2, 3
    ok = args([B, PV, ST, PV, EV], [[0], [4], [1, 2, 3]], [3, 1, 1])
    assert rc(ok)[0] == 0
    ok.slot_pv2[3] = 0
    r, msg = rc(ok)
    assert r == -1 and "PV parameter set" in msg      # two PVs on one parameter set
    r, msg = rc(args([B, PV, ST, PV, EV], [[0], [4], [1, 2]], [3, 1, 1]))
    assert r == -1 and "waves list" in msg
    r, msg = rc(args([B, PV, ST, PV, EV], [[0, 4], [1, 2, 3]], [3, 1, 1]))
    assert r == -1 and "wave of its own" in msg
    r, msg = rc(args([B, PV, ST, PV, EV], [[0], [4], [1, 2, 2]], [3, 1, 1]))
    assert r == -1 and "wave_slot" in msg
    bad = args([B, PV, ST, PV, EV], [[0], [4], [1, 2, 3]], [3, 2])
    bad.agent_sum[1] = 0
    r, msg = rc(bad)
    assert r == -1 and "one slot unless summed" in msg
    r, msg = rc(args([B, EV, EV], [[0], [1], [2]], [1, 1, 1]))
    assert r == -1 and "at most" in msg


MODELS = os.path.join(REPO, "tests", "data", "models_feeder.dss")


def test_dss_load_models_and_series_capacitor():
    """OpenDSS load models 1-8 and a series capacitor (tests/data/models_feeder.dss).
    Parity unpinned (no OpenDSS): the native build equals the oracle's
    independent NumPy build; a converged oracle solve satisfies the nodal
    equations; every element draws the power its model's law gives at its
    voltage (Feeder.LAWS); the series capacitor raises the voltage across it."""
    from oracle.pf_oracle import Feeder as OracleFeeder
    from powergridworld_amd.distribution_system.feeder import Feeder, load_feeder_spec
    spec = load_feeder_spec(MODELS)
    cap = [c for c in spec["capacitors"] if c["bus2"]]
    assert len(cap) == 1 and cap[0]["bus2"] == "B.1.2.3"
    m8 = [ld for ld in spec["loads"] if ld["model"] == 8][0]
    assert m8["zipv"] == [0.3, 0.3, 0.4, 0.5, 0.2, 0.3, 0.6]
    f, o = Feeder(spec), OracleFeeder(spec)
    assert f.node_names == o.node_names
    assert sorted(set(f.elem_model.tolist())) == [1, 3, 4, 5, 6, 7, 8]     # model 2: a shunt
    assert f.m == 3 + 1 + 1 + 3 + 1 + 1 + 3 + 3
    assert np.abs(f.Y - o.Y).max() / np.abs(o.Y).max() < 1e-12
    assert np.abs(f.Z - o.Z).max() / np.abs(o.Z).max() < 1e-10
    W, U0, G, V0 = f.reduce_rows([f.node_index["c.1"]])
    assert np.abs(W - o.W).max() / np.abs(o.W).max() < 1e-10
    kw = np.array([ld["kw"] for ld in spec["loads"]], float)
    kvar = np.array([ld["kvar"] for ld in spec["loads"]], float)
    V, it = o.solve(kw[None] * 1.3, kvar[None] * 1.3, tol=1e-13)
    W_ph = 1.3 * kw[o.elem_load] * 1000.0 / o.elem_nph
    var_ph = 1.3 * kvar[o.elem_load] * 1000.0 / o.elem_nph
    U = o.Cinc @ V[0]
    I = o.load_currents(U[None], W_ph[None], var_ph[None])[0]
    resid = np.abs(o.Y @ V[0] - (o.I_src - o.Cinc.T @ I)).max() / np.abs(o.I_src).max()
    assert resid < 1e-8
    S = U * np.conj(I)
    v = np.abs(U) / o.elem_vbase
    for k, li in enumerate(o.elem_load):
        ld = spec["loads"][li]
        md, vk = ld["model"], v[k]
        assert 0.9 < vk <= 1.05, (ld["name"], vk)
        P, Q = W_ph[k], var_ph[k]
        exp = {1: (P, Q), 3: (P, Q * vk ** 2), 4: (P * vk ** ld["cvrwatts"], Q * vk ** ld["cvrvars"]),
               5: (P * vk, Q * vk), 6: (P, Q), 7: (P, Q * vk ** 2)}
        if md == 8:
            z = ld["zipv"]
            exp[8] = (P * (z[0] * vk ** 2 + z[1] * vk + z[2]), Q * (z[3] * vk ** 2 + z[4] * vk + z[5]))
        if md in (1, 3, 6, 7) and vk <= 0.95:      # below Vminpu the constant-P part is constant Z
            continue
        np.testing.assert_allclose([S[k].real, S[k].imag], exp[md], rtol=1e-9, err_msg=ld["name"])
    i = f.node_index
    assert all(abs(V[0][o.idx["b.%d" % p]]) > abs(V[0][o.idx["a.%d" % p]]) for p in (1, 2, 3))


XFMR3 = os.path.join(REPO, "tests", "data", "xfmr3_feeder.dss")


def test_dss_three_winding_and_centre_tap_transformers():
    """3-winding and centre-tapped transformers (tests/data/xfmr3_feeder.dss).
    Parity unpinned (no OpenDSS): the native N-winding element equals the
    oracle's independent NumPy stamp; a converged solve satisfies the nodal
    equations; the unit's winding voltages sit at its turns ratios at no load
    (X at the 1.025 tap); the centre tap splits 240 V into two 120 V legs of
    opposite phase; the windings' complex powers balance up to the leakage
    losses (sum of S over all terminals = the losses, with P >= 0)."""
    from oracle.pf_oracle import Feeder as OracleFeeder
    from powergridworld_amd.distribution_system.feeder import Feeder, load_feeder_spec
    spec = load_feeder_spec(XFMR3)
    t3 = [t for t in spec["transformers"] if t["name"] == "t3"][0]
    assert len(t3["windings"]) == 3 and (t3["xhl"], t3["xht"], t3["xlt"]) == (4.5, 8.0, 3.5)
    assert [w["kva"] for w in t3["windings"]] == [1500.0, 1000.0, 500.0]
    f, o = Feeder(spec), OracleFeeder(spec)
    assert f.node_names == o.node_names
    assert np.abs(f.Y - o.Y).max() / np.abs(o.Y).max() < 1e-12
    assert np.abs(f.V0 - o.V0).max() / np.abs(o.V0).max() < 1e-12
    i = o.idx
    # no load: X at 0.48 kV x 1.025 over B's 4.16, T at B's; S legs 120 V, opposite phase
    pu0 = o.pu(o.V0)
    np.testing.assert_allclose(pu0[[i["x.1"], i["x.2"], i["x.3"]]] / pu0[i["b.1"]], 1.025, rtol=1e-6)
    np.testing.assert_allclose(abs(o.V0[i["s.1"]]) / abs(o.V0[i["a.1"]]), 0.12 / 2.4, rtol=1e-6)
    assert abs(o.V0[i["s.1"]] + o.V0[i["s.2"]]) < 1e-6 * abs(o.V0[i["s.1"]])
    kw = np.array([ld["kw"] for ld in spec["loads"]], float)
    kvar = np.array([ld["kvar"] for ld in spec["loads"]], float)
    V, it = o.solve(kw[None], kvar[None], tol=1e-13)
    W_ph = kw[o.elem_load] * 1000.0 / o.elem_nph
    var_ph = kvar[o.elem_load] * 1000.0 / o.elem_nph
    U = o.Cinc @ V[0]
    I = o.load_currents(U[None], W_ph[None], var_ph[None])[0]
    resid = np.abs(o.Y @ V[0] - (o.I_src - o.Cinc.T @ I)).max() / np.abs(o.I_src).max()
    assert resid < 1e-8
    # the loads draw their power inside their band (below Vminpu: constant Z)
    S = U * np.conj(I)
    inb = np.abs(U) / o.elem_vbase > 0.95
    assert inb.sum() >= 10
    np.testing.assert_allclose(S.real[inb], W_ph[inb], rtol=1e-9)
    np.testing.assert_allclose(S.imag[inb], var_ph[inb], rtol=1e-9)
    # T3's terminal power: its own stamp (an oracle feeder of the source and T3
    # alone; the source stamp sits on sourcebus only) at the solved voltages
    o2 = OracleFeeder(dict(spec, transformers=[t3], lines=[], loads=[], capacitors=[]))
    names = [nm for nm in o2.node_names if not nm.startswith("sourcebus")]
    a = [o2.idx[nm] for nm in names]
    Vt = V[0][[o.idx[nm] for nm in names]]
    S_in = Vt * np.conj(o2.Y[np.ix_(a, a)] @ Vt)          # into the unit per terminal
    loss = S_in.sum()
    p_through = S_in[:3].sum().real                        # from B (winding 1)
    assert p_through > 0 and 0 < loss.real < 0.02 * p_through


REGCTL = os.path.join(REPO, "tests", "data", "regctl_feeder.dss")


def test_regcontrol_model_woodbury_matches_rebuilt_network():
    """RegControl model (Feeder.regulators, tests/data/regctl_feeder.dss): the
    regulated phases' unit-tap admittances and the regulator nodes R give, through
    the Woodbury form the kernels use (Z(t) = Z0 - Z0 U K U^T Z0, K = (I + D S)^-1 D),
    the no-load voltages of the oracle's network rebuilt and re-inverted at the
    same taps; the oracle's control loop moves out-of-band regulators into band
    in whole steps (MaxTapChange respected).  Parity unpinned (no OpenDSS)."""
    from oracle.pf_oracle import Feeder as OracleFeeder
    from powergridworld_amd.distribution_system.feeder import Feeder, load_feeder_spec
    spec = load_feeder_spec(REGCTL)
    f, o = Feeder(spec), OracleFeeder(spec)
    reg = f.regulators()
    assert reg is not None and len(reg["ctrls"]) == 4 and len(reg["phases"]) == 6
    assert len(reg["nodes"]) == 12
    np.testing.assert_allclose(reg["taps0"], [1.0, 1.0125, 0.99375, 1.0])
    R, r = reg["nodes"], len(reg["nodes"])
    rng = np.random.default_rng(0)
    for _ in range(4):
        taps = reg["taps0"] + 0.00625 * rng.integers(-8, 9, size=4)
        D = np.zeros((r, r), complex)
        for ph in reg["phases"]:
            t = taps[ph["ctrl"]]
            t1 = t if ph["tap_winding"] == 1 else ph["tap1"]
            t2 = t if ph["tap_winding"] == 2 else ph["tap2"]
            Y = lambda a, b: np.array([[ph["A"] / a ** 2, ph["B"] / (a * b)], [ph["B"] / (a * b), ph["C"] / b ** 2]])
            D[np.ix_([ph["a"], ph["b"]], [ph["a"], ph["b"]])] += Y(t1, t2) - Y(ph["tap1"], ph["tap2"])
        K = np.linalg.solve(np.eye(r) + D @ reg["S"], D)
        V = f.V0 - f.Z[:, R] @ (K @ f.V0[R])
        ot = o.with_taps(list(taps))
        np.testing.assert_allclose(V, ot.V0, rtol=1e-9, atol=1e-9 * np.abs(ot.V0).max())
    kw = np.array([ld["kw"] for ld in spec["loads"]], float)
    kvar = np.array([ld["kvar"] for ld in spec["loads"]], float)
    V, it, tp, cp = o.solve_regulated(kw[None], kvar[None], reg["taps0"][None])
    assert cp[0] >= 2 and (tp[0] != reg["taps0"]).any()
    steps = (tp[0] - reg["taps0"]) / 0.00625
    np.testing.assert_allclose(steps, np.round(steps), atol=1e-9)
    # in band after the loop (the last pass moved nothing)
    _, moved = o.reg_control_pass(V[0], list(tp[0]))
    assert not moved


REGCTL2 = os.path.join(REPO, "tests", "data", "regctl2_feeder.dss")


def test_regcontrol_sample_options_model():
    """RegControl's Sample options (tests/data/regctl2_feeder.dss): Bus= puts
    the regulated bus's nodes into R as sensed nodes (no line-drop
    compensation; Vlimit then reads the winding's first phase), PTphase=max /
    min monitor every phase of a gang-operated unit, Vlimit and InverseTime
    reach the control records; the Woodbury model with the extra sensed nodes
    still gives the rebuilt network's voltages; the oracle's loop ends in band
    (or at Vlimit) at light load.  Parity unpinned (no OpenDSS)."""
    from powergridworld_amd import _lib
    from oracle.pf_oracle import Feeder as OracleFeeder
    from powergridworld_amd.distribution_system.feeder import Feeder, load_feeder_spec
    spec = load_feeder_spec(REGCTL2)
    f, o = Feeder(spec), OracleFeeder(spec)
    reg = f.regulators()
    R = reg["nodes"]
    name = lambda j: f.node_names[R[j]]
    c = {d["name"]: d for d in reg["ctrls"]}
    assert len(reg["phases"]) == 9 and len(R) == 21
    assert [name(j) for j in c["reg1"]["mon_node"]] == ["b3.1"] and c["reg1"]["ldc"] == 0
    assert name(c["reg1"]["vlim_node"]) == "rg60.1"
    assert c["reg2"]["ldc"] == 1 and c["reg2"]["vlimit"] == 126.5 and c["reg2"]["vlim_node"] == -1
    assert c["reg3"]["inverse_time"] == 1 and c["reg3"]["n_mon"] == 1
    assert c["regg"]["pick"] == _lib.REG_PICK_MAX and c["regg"]["n_mon"] == 3 and c["regg"]["ldc"] == 1
    assert [name(j) for j in c["regg"]["mon_node"]] == ["b5.1", "b5.2", "b5.3"]
    assert c["regh"]["pick"] == _lib.REG_PICK_MIN and c["regh"]["inverse_time"] == 1
    assert [name(j) for j in c["regh"]["mon_node"]] == ["b8.1", "b8.2", "b8.3"]
    assert c["regh"]["mon_phase"] == [6, 7, 8] and name(c["regh"]["vlim_node"]) == "b7.1"
    r = len(R)
    rng = np.random.default_rng(1)
    for _ in range(3):
        taps = reg["taps0"] + 0.00625 * rng.integers(-8, 9, size=len(reg["ctrls"]))
        D = np.zeros((r, r), complex)
        for ph in reg["phases"]:
            t = taps[ph["ctrl"]]
            t1 = t if ph["tap_winding"] == 1 else ph["tap1"]
            t2 = t if ph["tap_winding"] == 2 else ph["tap2"]
            Y = lambda a, b: np.array([[ph["A"] / a ** 2, ph["B"] / (a * b)], [ph["B"] / (a * b), ph["C"] / b ** 2]])
            D[np.ix_([ph["a"], ph["b"]], [ph["a"], ph["b"]])] += Y(t1, t2) - Y(ph["tap1"], ph["tap2"])
        K = np.linalg.solve(np.eye(r) + D @ reg["S"], D)
        V = f.V0 - f.Z[:, R] @ (K @ f.V0[R])
        ot = o.with_taps(list(taps))
        np.testing.assert_allclose(V, ot.V0, rtol=1e-9, atol=1e-9 * np.abs(ot.V0).max())
    kw = np.array([ld["kw"] for ld in spec["loads"]], float)
    kvar = np.array([ld["kvar"] for ld in spec["loads"]], float)
    V, it, tp, cp = o.solve_regulated(0.5 * kw[None], 0.5 * kvar[None], reg["taps0"][None])
    assert 2 <= cp[0] < 15 and (tp[0] != reg["taps0"]).any()
    _, moved = o.reg_control_pass(V[0], list(tp[0]))
    assert not moved


def test_regcontrol_options_oracle_semantics():
    """The oracle's Sample options on regctl2_feeder.dss, from chosen taps:
    Vlimit forces Reg2 down while its local voltage is above the limit
    (whatever its compensated voltage asks) and the control loop ends at or
    below it; the options reach the oracle's control records."""
    from oracle.pf_oracle import Feeder as OracleFeeder
    from powergridworld_amd.distribution_system.feeder import load_feeder_spec
    spec = load_feeder_spec(REGCTL2)
    o = OracleFeeder(spec)
    ctrls = o.reg_controls()
    names = [t["name"] for t, _ in ctrls]
    kw = np.array([ld["kw"] for ld in spec["loads"]], float) * 0.5
    kvar = np.array([ld["kvar"] for ld in spec["loads"]], float) * 0.5
    taps = [1.0, 1.1, 0.99375, 1.0, 1.0]                 # Reg2 at its top tap: local voltage above Vlimit
    f = o.with_taps(taps)
    V, _ = f.solve(kw[None], kvar[None], tol=1e-12)
    V = V[0]
    t2, c2 = ctrls[names.index("reg2")]
    a, b = o._reg_nodes(t2, 0)
    assert abs(V[b]) / c2["ptratio"] > c2["vlimit"]
    # Reg2 acts (down, toward the limit) unless an inverse-time control's
    # shorter delay claims this pass (only the nearest-delay actions act)
    out, moved = o.reg_control_pass(V, taps)
    assert moved
    g2 = names.index("reg2")
    if out[g2] != taps[g2]:
        assert out[g2] < taps[g2]
    else:
        assert any(out[g] != taps[g] and ctrls[g][1]["inverse"] for g in range(len(ctrls)))
    # the loop from there ends with Reg2's local voltage at or below the limit
    Vl, _, tp, _ = o.solve_regulated(kw[None], kvar[None], np.array(taps)[None])
    assert abs(Vl[0][b]) / c2["ptratio"] <= c2["vlimit"] + 1e-9
    assert o.reg_controls()[names.index("regh")][1]["bus"] == "b8"
    assert ctrls[names.index("reg3")][1]["inverse"] and not ctrls[names.index("reg1")][1]["inverse"]


def test_regcontrol_inverse_time_vlimit_only_trigger():
    """InverseTime with Vlimit the only trigger (|Vreg - V| = 0): the oracle's
    delay is Delay / 0 = +inf, as k_reg_control's IEEE division gives (ADVICE
    r05: it raised ZeroDivisionError), and the tap still moves down toward the
    limit."""
    from oracle.pf_oracle import Feeder as OracleFeeder
    from powergridworld_amd.distribution_system.feeder import load_feeder_spec
    spec = load_feeder_spec(REGCTL2)
    o = OracleFeeder(spec)
    ctrls = o.reg_controls()
    names = [t["name"] for t, _ in ctrls]
    t, c = ctrls[names.index("reg3")]
    kw = np.array([ld["kw"] for ld in spec["loads"]], float) * 0.5
    kvar = np.array([ld["kvar"] for ld in spec["loads"]], float) * 0.5
    taps = [1.0, 1.0, 1.0, 1.0, 1.0]
    V = o.with_taps(taps).solve(kw[None], kvar[None], tol=1e-12)[0][0]
    a, b = o._reg_nodes(t, 0)
    c2 = dict(c, R=0.0, X=0.0, bus="", ptphase=1, inverse=True)
    vc = abs(V[a if c2["winding"] == 1 else b] / c2["ptratio"])
    c2["vreg"], c2["vlimit"] = vc, 0.99 * vc                 # dv = 0 exactly, local voltage above the limit
    o.reg_controls = lambda: [(t, c2)]
    out, moved = o.reg_control_pass(V, [taps[names.index("reg3")]])
    assert moved and out[0] < taps[names.index("reg3")]


def test_regcontrol_refuses_unsimulated_options(tmp_path):
    """Reversible regulators and PTphase=avg stay refused, loudly."""
    from powergridworld_amd.distribution_system.feeder import Feeder, load_feeder_spec
    txt = open(REGCTL2).read()
    for old, bad in (("maxtapchange=4 inversetime=yes", "maxtapchange=4 inversetime=yes reversible=yes"),
                     ("ptphase=max", "ptphase=avg")):
        assert old in txt
        fn = tmp_path / "bad.dss"
        fn.write_text(txt.replace(old, bad, 1))
        with pytest.raises(NotImplementedError):
            Feeder(load_feeder_spec(str(fn))).regulators()


def test_regcontrol_bus_without_nodes_off_phase_1_refused(tmp_path):
    """Bus= with no node numbers on a single-phase regulator of phase 2: which
    node OpenDSS senses there is unpinned, so it is refused; the
    same control with the node named is accepted and senses that node."""
    from powergridworld_amd.distribution_system.feeder import Feeder, load_feeder_spec
    txt = open(REGCTL2).read()
    old = "New RegControl.Reg2 transformer=Reg2 winding=2 vreg=123 band=2 ptratio=20 ctprim=700 R=3 X=6 vlimit=126.5"
    assert old in txt
    fn = tmp_path / "bus_nonodes.dss"
    fn.write_text(txt.replace(old, old + " bus=B3", 1))
    with pytest.raises(NotImplementedError):
        Feeder(load_feeder_spec(str(fn))).regulators()
    fn2 = tmp_path / "bus_node2.dss"
    fn2.write_text(txt.replace(old, old + " bus=B3.2", 1))
    f = Feeder(load_feeder_spec(str(fn2)))
    reg = f.regulators()
    assert reg is not None and f.node_index["b3.2"] in [int(x) for x in np.asarray(reg["nodes"])]


def test_checkpoint_walk_restores_in_place():
    """checkpoint.state_dict / load_state_dict on a stand-in object tree (CPU
    tensors): tensors restored in place (identity kept), a view restored
    through its base, generator states and clocks reset, caches and version
    counters left alone."""
    import torch
    from powergridworld_amd import checkpoint

    class Part:                      # (module powergridworld_amd: walked)
        pass
    Part.__module__ = "powergridworld_amd.test_stub"
    env = Part()
    env.time_index, env.tables_version, env.step_cache = 3, 7, {"k": 1}
    env.soc = torch.arange(4.0)
    env.obs_view = env.soc.view(2, 2).t()
    env.gen = torch.Generator().manual_seed(1)
    env.sub = Part()
    env.sub.x = torch.ones(3)
    env.sub.flags = {"a": torch.zeros(2), "n": 5}
    sd = checkpoint.state_dict(env)
    soc_id = id(env.soc)
    env.soc += 10
    env.sub.x.mul_(3)
    env.sub.flags["a"].fill_(9)
    env.time_index, env.tables_version = 9, 8
    r1 = torch.rand(2, generator=env.gen)
    checkpoint.load_state_dict(env, sd)
    assert id(env.soc) == soc_id and torch.equal(env.soc, torch.arange(4.0))
    assert torch.equal(env.sub.x, torch.ones(3)) and torch.equal(env.sub.flags["a"], torch.zeros(2))
    assert env.time_index == 3 and env.tables_version == 8          # (version counters untouched)
    assert torch.equal(torch.rand(2, generator=env.gen), r1)
    assert "step_cache" not in " ".join(sd)


def test_opendss_solver_reading_options_refused():
    """The two readings of the snap solve this build cannot confirm without
    OpenDSS are options with their own constraints:
    yprim='step' (H1) and snap_start='previous' are OpenDSS-rule readings, and
    H1 starts from the direct solution; unknown values are refused."""
    from powergridworld_amd.distribution_system.opendss import OpenDSSSolver
    feeder, shape = "ieee_13_dss/IEEE13Nodeckt.dss", "ieee_13_dss/annual_hourly_load_profile.csv"
    for kw in (dict(yprim="nope"), dict(yprim="step", convergence="exact"),
               dict(yprim="step", snap_start="previous"), dict(snap_start="later"),
               dict(snap_start="previous", convergence="exact")):
        with pytest.raises(ValueError):
            OpenDSSSolver(feeder, shape, **kw)
