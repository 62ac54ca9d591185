"""Synthetic exogenous building data (test infrastructure).

The reference's ``gridworld/agents/buildings/data/exogenous_data.csv`` is a
missing large blob, so every party -- the reference run by
``make_golden.py``, the oracle and the product tests -- is fed the same
synthetic frame, defined in SURVEY.md 8(d):

    T_oa      = 24 + 8 sin(2 pi (t/288 - 0.3))
    Q_solar_z = max(0, 3 sin(2 pi (t/288 - 0.25))) + 0.1 U
    Q_cool_z  = -2 - U
    Q_int_z   = 1 + 0.5 U

with t = five-minute slot of the day and U ~ U[0,1) from
``numpy.random.default_rng(seed)`` drawn as three (rows, 5) blocks in the
order solar, cool, int.  Columns follow the reference's regex lookups
(``five_zone_rom_env.py:55-57,140-144``).
"""
import numpy as np
import pandas as pd

DEFAULT_START = "2020-08-11 00:00:00"
DEFAULT_END = "2020-08-14 00:00:00"


def synthetic_exogenous_frame(start=DEFAULT_START, end=DEFAULT_END, seed=0):
    idx = pd.date_range(pd.Timestamp(start), pd.Timestamp(end), freq="5min")
    n = len(idx)
    t = ((idx.hour * 60 + idx.minute) // 5).values.astype(np.float64)
    rng = np.random.default_rng(seed)
    u_solar = rng.random((n, 5))
    u_cool = rng.random((n, 5))
    u_int = rng.random((n, 5))
    cols = {"T_oa": 24.0 + 8.0 * np.sin(2 * np.pi * (t / 288.0 - 0.3))}
    solar = np.maximum(0.0, 3.0 * np.sin(2 * np.pi * (t / 288.0 - 0.25)))
    for z in range(5):
        cols["Q_solar_%d" % z] = solar + 0.1 * u_solar[:, z]
    for z in range(5):
        cols["Q_cool_%d" % z] = -2.0 - u_cool[:, z]
    for z in range(5):
        cols["Q_int_%d" % z] = 1.0 + 0.5 * u_int[:, z]
    return pd.DataFrame(cols, index=idx)
