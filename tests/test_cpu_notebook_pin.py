"""External pin of the feeder model on the reference's own OpenDSS output.

The reference holds no power-flow fixture, but its single-component demo
notebook (examples/envs/multiagent-single-component.ipynb, cells 2-6) plots
the per-step minimum node voltage of one random-policy episode solved by
OpenDSS: three EV-charging agents (100 vehicles each, multiplier 2, 7 kW,
5-minute steps) on bus 675c, IEEE-13 at system_load_rescale_factor 0.8,
2020-08-12 00:00 -> 2020-08-13 00:00.  tools/digitize_notebook_plots.py turned
that panel into tests/golden/notebook_minv.npz: per step the pu band the
plotted line covers (about 0.00033 pu per pixel).

The actions were random, so the check is an envelope: at each step the three
agents together draw some P in [0, 3 * 2 * 7 kW * 5/60 h * parked vehicles]
at 675c (ev_charging_env.py:186-187 parked test, :208-255 charge and
vehicle_multiplier; the kWh-per-step value goes to the power flow as kW), so
the plotted minimum must lie between the min and the max over that P range of
the model's minimum node voltage (all nodes, as `df.min(axis=1)`).  The min
over P is not monotone (load on phase c lifts the phase that holds the
minimum), so P is swept.  The band spans +-0.8 px about the step's x, which
reaches the line segments to both neighbours, hence the neighbour union.

What it pins: the feeder (Y, transformer and regulator taps, load models and
placement), the hour-of-year -> loadshape mapping and the rescale factor.
Controls: a 2.5 % rescale error or a one-hour shift puts tens of steps out
by several pixels.  What it does not pin: the stopping rule -- the exact fixed
point and the OpenDSS snap iterate differ by ~1e-5 pu, far below a pixel.
"""
import os

import numpy as np
import pandas as pd
import pytest

from oracle.pf_oracle import BatchedPF
from oracle.pgw_oracle import EVOracle

GOLD = os.path.join(os.path.dirname(__file__), "golden", "notebook_minv.npz")
T0 = pd.Timestamp("2020-08-12 00:00")
AGENTS, MULT, RATE_KW, MPS = 3, 2.0, 7.0, 5
FRACTIONS = np.linspace(0.0, 1.0, 41)
TOL_PX = 0.5                 # digitisation: the band edges are antialiased pixels


def _data():
    g = np.load(GOLD)
    return g["single_minutes"], g["single_lo"], g["single_hi"], float(g["single_pu_per_px"])


def _pmax(minutes):
    ev = EVOracle(1, num_vehicles=100, minutes_per_step=MPS, max_charge_rate_kw=RATE_KW,
                  peak_threshold=250., vehicle_multiplier=MULT, rescale_spaces=False)
    # vehicles parked at any time the step's band reaches (two steps each way)
    parked = np.array([max(((ev.start <= t) & (t <= ev.endp)).sum() for t in m + MPS * np.arange(-2, 3))
                       for m in minutes])
    return AGENTS * MULT * RATE_KW * MPS / 60.0 * parked


def _outside_px(rescale=0.8, shift_h=0, semantics="opendss", idx=None):
    minutes, lo, hi, px = _data()
    if idx is not None:
        minutes, lo, hi = minutes[idx], lo[idx], hi[idx]
    pmax = _pmax(minutes)
    pf = BatchedPF(system_load_rescale_factor=rescale, semantics=semantics)
    t0 = T0 + pd.Timedelta(hours=shift_h)
    v = np.array([pf.calculate(t0 + pd.Timedelta(minutes=float(m)), {"675c": FRACTIONS * p}, None,
                               K=len(FRACTIONS)).min(1) for m, p in zip(minutes, pmax)])
    nb = lambda x, f: np.array([f(x[max(k - 1, 0):k + 2]) for k in range(len(x))])
    top, bot = nb(v.max(1), np.max), nb(v.min(1), np.min)
    return np.maximum((lo - top) / px, (bot - hi) / px)


def test_digitised_fixture_shape():
    minutes, lo, hi, px = _data()
    assert len(minutes) >= 280 and np.all(np.diff(minutes) > 0)
    assert np.all(hi >= lo) and np.all((lo > 0.93) & (hi < 0.99))
    assert 2e-4 < px < 5e-4


@pytest.mark.parametrize("semantics", ["opendss", "exact"])
def test_notebook_min_voltage_inside_model_envelope(semantics):
    out = _outside_px(semantics=semantics)
    assert out.max() <= TOL_PX, (out.max(), np.nonzero(out > TOL_PX)[0])


def test_notebook_zero_load_steps_are_point_pins():
    """Steps with no vehicle parked (about 21:30 - 22:55): envelope = one value."""
    minutes, lo, hi, px = _data()
    idx = np.nonzero(_pmax(minutes) == 0.0)[0]
    assert len(idx) >= 10
    pf = BatchedPF(system_load_rescale_factor=0.8, semantics="opendss")
    v = np.array([pf.calculate(T0 + pd.Timedelta(minutes=float(m))).min() for m in minutes[idx]])
    # inside the step's band (neighbour segments can widen it at an hour edge)
    assert np.all(v >= lo[idx] - TOL_PX * px) and np.all(v <= hi[idx] + TOL_PX * px)


@pytest.mark.parametrize("wrong", [dict(rescale=0.78), dict(rescale=0.82), dict(shift_h=1), dict(shift_h=-1)])
def test_notebook_pin_rejects_wrong_models(wrong):
    out = _outside_px(**wrong)
    assert (out > 1.0).sum() >= 10 and out.max() > 2.0, out.max()
