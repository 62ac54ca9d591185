"""Convert the reference's DATA assets into this package's own formats.

Runs only in the build container (it reads ``/root/reference``); its outputs
under ``powergridworld_amd/data/`` are committed, so nothing here ever runs on
the GPU box.  Only data is converted -- no reference source is copied.

* PV max-power profiles  (``gridworld/agents/pv/profiles/*.csv``)       -> pv_profiles.npz
* EV vehicle schedule    (``gridworld/agents/vehicles/vehicles.csv``)   -> vehicles.npz
* IEEE-13 hourly loadshape (``distribution_system/data/ieee_13_dss/annual_hourly_load_profile.csv``)
                                                                         -> loadshape_8760.npy
* 5-zone ROM state-space model (``gridworld/agents/buildings/data/state_space_model.p``)
                                                                         -> state_space_model.json
* Home-Steward scenario, vehicles, device profiles, grid cost   -> hs_data.json

The pickle is NOT unpickled: it is walked opcode-by-opcode with
``pickletools.genops`` (which executes nothing) and the raw little-endian
array payloads are decoded by hand.  The result is cross-checked against the
reference's own text dump ``state_space_model.json`` (written by
``gridworld/agents/buildings/test.py:1-8``).

Data license: PowerGridworld is BSD-3-Clause (reference ``LICENSE:1-3``);
see ``powergridworld_amd/data/NOTICE``.
"""
import ast
import json
import os
import pickletools
import re

import numpy as np
import pandas as pd

REF = "/root/reference/gridworld"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                   "powergridworld_amd", "data")

SS_KEYS = ["ss_A", "ss_B", "ss_C", "ss_D", "ss_K", "input_sel_list",
           "mean_inputs", "mean_output", "neighbors", "x_k"]
INT_KEYS = {"ss_C", "ss_D", "input_sel_list", "mean_inputs"}


def extract_state_space_model(path):
    """Walk the pickle's opcodes (no execution) and recover the 5 zone dicts."""
    data = open(path, "rb").read()
    zones, cur, key = [], None, None
    memo, last_str = [], None   # memo index -> string (keys are memoized after first use)
    for op, arg, _ in pickletools.genops(data):
        if op.name == "MEMOIZE":
            memo.append(last_str)
            last_str = None
            continue
        if op.name in ("BINGET", "LONG_BINGET") and memo[arg] in SS_KEYS:
            op_name, arg = "SHORT_BINUNICODE", memo[arg]
        else:
            op_name = op.name
        last_str = arg if op_name in ("SHORT_BINUNICODE", "BINUNICODE") else None
        if op_name == "EMPTY_DICT":
            cur = {}
            zones.append(cur)
            key = None
        elif op_name in ("SHORT_BINUNICODE", "BINUNICODE") and arg in SS_KEYS:
            key = arg
            if key == "neighbors":
                cur[key] = []
        elif op_name in ("SHORT_BINBYTES", "BINBYTES") and key is not None \
                and key != "neighbors" and len(arg) >= 8:
            dt = "<i8" if key in INT_KEYS else "<f8"
            cur[key] = np.frombuffer(arg, dtype=dt).tolist()
            key = None
        elif op_name in ("BININT1", "BININT", "BININT2") and key == "neighbors":
            cur["neighbors"].append(int(arg))
        elif op_name == "APPENDS" and key == "neighbors":
            key = None
    return zones


def check_against_text_dump(zones, path):
    txt = open(path).read()
    txt = re.sub(r"array\(", "(", txt)
    dump = ast.literal_eval(txt)
    assert len(dump) == len(zones) == 5
    for z, (a, b) in enumerate(zip(zones, dump)):
        for k in SS_KEYS:
            va = np.ravel(np.asarray(a[k], dtype=float))
            vb = np.ravel(np.asarray(b[k], dtype=float))
            assert va.shape == vb.shape, (z, k, va, vb)
            assert np.allclose(va, vb, rtol=1e-7, atol=0), (z, k, va, vb)


def main():
    os.makedirs(OUT, exist_ok=True)

    # PV profiles: the reference reads column 0 of each CSV (pv_profile_env.py:274).
    prof = {}
    for name in ["pv_profile", "constant", "off-peak", "pv_profile_hs"]:
        p = os.path.join(REF, "agents/pv/profiles", name + ".csv")
        prof[name] = pd.read_csv(p).values[:, 0].astype(np.float64)
    np.savez(os.path.join(OUT, "pv_profiles.npz"), **prof)

    # Vehicle schedule (ev_charging_env.py:70-76 reads and rounds these).
    df = pd.read_csv(os.path.join(REF, "agents/vehicles/vehicles.csv"))
    np.savez(os.path.join(OUT, "vehicles.npz"),
             start_time_min=df["start_time_min"].values.astype(np.int64),
             end_time_park_min=df["end_time_park_min"].values.astype(np.int64),
             energy_required_kwh=df["energy_required_kwh"].values.astype(np.float64))

    # IEEE-13 annual hourly loadshape (opendss.py:44 uses np.genfromtxt).
    ls = np.genfromtxt(os.path.join(
        REF, "distribution_system/data/ieee_13_dss/annual_hourly_load_profile.csv"))
    np.save(os.path.join(OUT, "loadshape_8760.npy"), ls.astype(np.float64))

    # Building state-space model.
    zones = extract_state_space_model(
        os.path.join(REF, "agents/buildings/data/state_space_model.p"))
    check_against_text_dump(
        zones, os.path.join(REF, "agents/buildings/data/state_space_model.json"))
    with open(os.path.join(OUT, "state_space_model.json"), "w") as f:
        json.dump({"zones": zones}, f, indent=1)
    # Home-Steward data: the shipped house scenario (scenarios/data/env_config.json,
    # read by heterogeneous_hs.py:45-57), its grid-cost series, and the default
    # vehicle / device profiles the HS components fall back to.
    with open(os.path.join(REF, "scenarios/data/env_config.json")) as f:
        hs_cfg = json.load(f)
    veh = pd.read_csv(os.path.join(REF, "agents/vehicles/vehicles_hs.csv"))
    dev = pd.read_csv(os.path.join(REF, "agents/devices/data/devices_profile_hs.csv"))
    gc = pd.read_csv(os.path.join(REF, "scenarios/data/grid_cost.csv"))
    hs = {"env_config": hs_cfg,
          "vehicles_hs": json.loads(veh.to_json(orient="split")),
          "devices_profile_hs": {c: dev[c].astype(float).tolist() for c in dev.columns},
          "grid_cost": {"time": gc["time"].tolist(), "grid_cost": gc["grid_cost"].astype(float).tolist()}}
    with open(os.path.join(OUT, "hs_data.json"), "w") as f:
        json.dump(hs, f)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
