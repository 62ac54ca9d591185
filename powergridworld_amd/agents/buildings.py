"""Batched five-zone reduced-order building (reference:
gridworld/agents/buildings/five_zone_rom_env.py, five_zone_rom_dynamics.py,
obs_space.py, defaults.py).

The per-zone Kalman-filtered LTI model and the HVAC power/comfort reward run
in pgw_building_reset / pgw_building_step, one thread per env; x_k lives in a
[5, N] device tensor and -- exactly like the reference, which never
re-initialises ``self.models`` -- persists across ``reset()``.
"""
import json
import os
from collections import OrderedDict
from typing import Tuple, Union

import numpy as np
import pandas as pd
import torch

from powergridworld_amd import _lib, spaces
from powergridworld_amd.base import ComponentEnv, as_action, as_env_tensor, oob_poll, register_env
from powergridworld_amd.log import logger
from powergridworld_amd.utils import maybe_rescale_box_space

DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")

MAX_FLOW_RATE = [2.2, 2.2, 2.2, 2.2, 3.2]      # five_zone_rom_env.py:22-26
MIN_FLOW_RATE = [.22, .22, .22, .22, .32]
MAX_TOTAL_FLOW_RATE = 10.0
MAX_DISCHARGE_TEMP = 16.0
MIN_DISCHARGE_TEMP = 10.0
DEFAULT_COMFORT_BOUNDS = (22., 28.)

# obs_space.py:9-48
ZONE_TEMP_BOUNDS = (16., 40.)
DEFAULT_OBS_CONFIG = OrderedDict({
    "zone_temp": ZONE_TEMP_BOUNDS,
    "zone_upper_viol": (-10., 10.),
    "zone_lower_viol": (-10., 10.),
    "comfort_lower": (20., 23.),
    "comfort_upper": (23., 26.),
    "outdoor_temp": (0., 56.),
    "p_setpoint": (0., 200.),
    "p_consumed": (0., 200.),
    "time_of_day": (0., 1.),
    "bus_voltage": (0.90, 1.10),
    "min_voltage": (0.90, 1.10),
    "max_voltage": (0.90, 1.10),
})
MULTIZONE_KEYS = ["zone_temp", "zone_upper_viol", "zone_lower_viol"]

# defaults.py:2-10
default_obs_config = {
    "zone_upper_viol": (-10., 10.),
    "zone_lower_viol": (-10., 10.),
    "comfort_lower": (20., 25.),
    "comfort_upper": (25., 30),
    "outdoor_temp": (0., 56.),
    "p_consumed": (0., 100.),
    "time_of_day": (0., 1.),
}

# reference state-dict order (five_zone_rom_env.py:246-262) -> kernel variable ids
_STATE_ORDER = (["zone_temp_%d" % z for z in range(5)] + ["zone_upper_viol_%d" % z for z in range(5)]
                + ["zone_lower_viol_%d" % z for z in range(5)]
                + ["comfort_lower", "comfort_upper", "outdoor_temp", "p_consumed", "time_of_day",
                   "bus_voltage", "min_voltage", "max_voltage", "p_setpoint"])
_VAR_ID = {k: i for i, k in enumerate(_STATE_ORDER)}


def make_obs_space(num_zones: int, config: dict):
    """obs_space.py:66-101: bounds in DEFAULT_OBS_CONFIG order."""
    for key in config:
        assert key in DEFAULT_OBS_CONFIG, "invalid key {}".format(key)
    lo, hi, labels = [], [], []
    for key in [k for k in DEFAULT_OBS_CONFIG if k in config]:
        if key in MULTIZONE_KEYS:
            lo += [config[key][0]] * num_zones
            hi += [config[key][1]] * num_zones
            labels.extend([key + "_" + str(i) for i in range(num_zones)])
        else:
            lo.append(config[key][0])
            hi.append(config[key][1])
            labels.append(key)
    box = spaces.Box(np.array(lo, dtype=float), np.array(hi, dtype=float), dtype=np.float64)
    return box, labels


def synthetic_exogenous_data(start="2020-08-11 00:00:00", end="2020-08-14 00:00:00", seed=0):
    """Synthetic stand-in for the reference's missing exogenous_data.csv
    (.MISSING_LARGE_BLOBS:1); formula of SURVEY.md 8(d):
    T_oa = 24 + 8 sin(2 pi (t/288 - 0.3)); Q_solar = max(0, 3 sin(2 pi (t/288 - 0.25))) + 0.1 U;
    Q_cool = -2 - U; Q_int = 1 + 0.5 U, t = 5-min slot of the day."""
    idx = pd.date_range(pd.Timestamp(start), pd.Timestamp(end), freq="5min")
    n = len(idx)
    t = ((idx.hour * 60 + idx.minute) // 5).values.astype(np.float64)
    rng = np.random.default_rng(seed)
    u_solar, u_cool, u_int = rng.random((n, 5)), rng.random((n, 5)), rng.random((n, 5))
    cols = {"T_oa": 24.0 + 8.0 * np.sin(2 * np.pi * (t / 288.0 - 0.3))}
    solar = np.maximum(0.0, 3.0 * np.sin(2 * np.pi * (t / 288.0 - 0.25)))
    for z in range(5):
        cols["Q_solar_%d" % z] = solar + 0.1 * u_solar[:, z]
    for z in range(5):
        cols["Q_cool_%d" % z] = -2.0 - u_cool[:, z]
    for z in range(5):
        cols["Q_int_%d" % z] = 1.0 + 0.5 * u_int[:, z]
    return pd.DataFrame(cols, index=idx)


def load_state_space_model():
    with open(os.path.join(DATA_DIR, "state_space_model.json")) as f:
        return json.load(f)["zones"]


def load_data(start_time=None, end_time=None, exogenous_data=None):
    """five_zone_rom_env.py:30-52.  ``exogenous_data``: DataFrame, CSV path, or None
    (-> $PGW_EXOGENOUS_CSV, data/exogenous_data.csv, else the synthetic frame)."""
    if exogenous_data is None:
        path = os.environ.get("PGW_EXOGENOUS_CSV", os.path.join(DATA_DIR, "exogenous_data.csv"))
        exogenous_data = path if os.path.exists(path) else None
    if exogenous_data is None:
        df = synthetic_exogenous_data()
    elif isinstance(exogenous_data, pd.DataFrame):
        df = exogenous_data
    else:
        df = pd.read_csv(exogenous_data, index_col=0)
        df.index = pd.DatetimeIndex(df.index)
    start_time = pd.Timestamp(start_time) if start_time else df.index[0]
    end_time = pd.Timestamp(end_time) if end_time else df.index[-1]
    _df = df.loc[start_time:end_time]
    if _df is None or len(_df) == 0:
        raise ValueError(
            f"start and/or end times ({start_time}, {end_time}) " +
            "resulted in empty dataframe.  First and last indices are " +
            f"({df.index[0]}, {df.index[-1]}), choose values in this range.")
    return _df, load_state_space_model()


@register_env
class FiveZoneROMEnv(ComponentEnv):
    """Five-zone ROM building; action = 5 zone flows + discharge temperature."""

    fused_kind = None           # only the ThermalEnergy reward is fused
    reward_kind = "viol"
    supported_dtypes = (torch.float64, torch.float32)    # fp32: pgw_building_*_f32

    def __init__(self, name: str = None, obs_config: dict = None,
                 start_time: Union[str, pd.Timestamp] = None, end_time: Union[str, pd.Timestamp] = None,
                 comfort_bounds=None, zone_temp_init: np.ndarray = None, max_episode_steps: int = None,
                 rescale_spaces: bool = True, exogenous_data=None, num_envs: int = 1, device=None,
                 dtype=None, **kwargs):
        super().__init__(name=name, num_envs=num_envs, device=device, dtype=dtype)
        self.rescale_spaces = rescale_spaces
        self.num_zones = 5
        self.obs_config = obs_config if obs_config is not None else default_obs_config
        self.zone_temp_init = (np.array(zone_temp_init, dtype=np.float64).copy()
                               if zone_temp_init is not None else 27. * np.ones(5))
        self.df, self.models = load_data(start_time, end_time, exogenous_data)
        max_steps = self.df.shape[0] - 3                                    # :97
        self.max_episode_steps = max_steps if max_episode_steps is None else min(max_episode_steps, max_steps)
        self.comfort_bounds = comfort_bounds if comfort_bounds is not None else DEFAULT_COMFORT_BOUNDS
        self.act_low = np.array(MIN_FLOW_RATE + [MIN_DISCHARGE_TEMP])
        self.act_high = np.array(MAX_FLOW_RATE + [MAX_DISCHARGE_TEMP])
        self._action_space = spaces.Box(low=self.act_low, high=self.act_high, dtype=np.float64)
        self.action_space = maybe_rescale_box_space(self._action_space, rescale_spaces)
        self.comfort_bounds_df = self.make_comfort_bounds_df()
        self._observation_space, self._obs_labels = make_obs_space(self.num_zones, self.obs_config)
        self.observation_space = maybe_rescale_box_space(self._observation_space, rescale_spaces)
        self._build_tables()
        self.params = self._make_params()
        self._bind_oob(self.oob_count)
        n = self.num_envs
        x0 = np.array([float(np.ravel(m["x_k"])[0]) for m in self.models])
        self.x = torch.tensor(np.tile(x0[:, None], (1, n)), dtype=self.dtype, device=self.device)
        self.p_consumed = torch.zeros(n, dtype=self.dtype, device=self.device)
        self._reward_state = torch.zeros(n, dtype=self.dtype, device=self.device)
        self._reward_out = torch.zeros(n, dtype=self.dtype, device=self.device)
        self._obs = self._new_obs(len(self._obs_labels))
        self.time_index = None

    @property
    def time(self):
        """Timestamp of the current exogenous row (five_zone_rom_env.py:188,219)."""
        return None if self.time_index is None else self.df.index[self.time_index]

    # ---------------------------------------------------------------- setup
    def make_comfort_bounds_df(self) -> pd.DataFrame:
        data = np.zeros((self.df.shape[0], 2))
        if isinstance(self.comfort_bounds, tuple):
            data[:, 0], data[:, 1] = self.comfort_bounds[0], self.comfort_bounds[1]
        else:
            cb = np.asarray(self.comfort_bounds)
            data[:, 0] = cb[:data.shape[0], 0]
            data[:, 1] = cb[:data.shape[0], 1]
        return pd.DataFrame(data, columns=["temp_lb", "temp_ub"], index=self.df.index)

    def _build_tables(self):
        cols = list(self.df.columns)
        pick = lambda pre: self.df[[c for c in cols if c.startswith(pre)]].values.astype(np.float64)
        self._T_oa = pick("T_oa")[:, 0]
        self._q_solar, self._q_cool, self._q_int = pick("Q_solar"), pick("Q_cool_"), pick("Q_int")
        self._cb = self.comfort_bounds_df.values.astype(np.float64)
        self._exo = []
        for t in range(len(self.df)):
            ex = _lib.BuildingExo()
            ex.T_oa = self._T_oa[t]
            for z in range(5):
                ex.q_solar[z] = self._q_solar[t, z]
                ex.q_int[z] = self._q_int[t, z]
                ex.q_cool[z] = self._q_cool[t, z]
            ex.comfort_lb, ex.comfort_ub = self._cb[t, 0], self._cb[t, 1]
            ex.time_of_day = 1. * t / self.max_episode_steps                # :253
            self._exo.append(ex)

    def _make_params(self):
        p = _lib.BuildingParams()
        m = self.models
        for z in range(5):
            p.A[z] = float(np.ravel(m[z]["ss_A"])[0])
            b32 = np.asarray(np.ravel(m[z]["ss_B"]), dtype=np.float64).astype(np.float32)   # dynamics.py:51
            for j in range(4):
                p.B[z][j] = float(b32[j])
                p.sel[z][j] = int(np.ravel(m[z]["input_sel_list"])[j]) - 1
                p.nbr[z][j] = int(m[z]["neighbors"][j])
            p.K[z] = float(np.ravel(m[z]["ss_K"])[0])
            p.C[z] = float(np.ravel(m[z]["ss_C"])[0])
            p.mean[z] = float(np.ravel(m[z]["mean_output"])[0])
            p.T_init[z] = float(self.zone_temp_init[z])
        for j in range(6):
            p.act_low[j], p.act_high[j] = self.act_low[j], self.act_high[j]
        # values in state-dict order, bounds in make_obs_space order (:265-270)
        vals = [k for k in _STATE_ORDER if k in self._obs_labels]
        if len(vals) > _lib.BLD_MAX_OBS:
            raise ValueError("too many building observations")
        p.n_obs = len(vals)
        for j, k in enumerate(vals):
            p.obs_var[j] = _VAR_ID[k]
            p.obs_low[j] = self._observation_space.low[j]
            p.obs_high[j] = self._observation_space.high[j]
        p.alpha = 0.2                                                         # :318
        p.rescale = int(bool(self.rescale_spaces))
        return p

    def _adopt(self, x=None, obs=None):
        if x is not None:
            x.copy_(self.x)
            self.x = x
        if obs is not None:
            self._obs = obs
        self._bufv += 1
        ComponentEnv._bufv_gen += 1

    def _ext(self, kw):
        n = self.num_envs
        keep = []
        ext = _lib.BuildingExt()
        for key in ("bus_voltage", "min_voltage", "max_voltage", "p_setpoint"):
            v = kw.get(key)
            if v is not None:
                if isinstance(v, (list, tuple)):
                    raise ValueError("%s must be a scalar per env (3-phase bus lists are not "
                                     "supported as building observations)" % key)
                t = as_env_tensor(v, n, self.device, key)
                keep.append(t)
                setattr(ext, key, t.data_ptr())
        return ext, keep

    # ---------------------------------------------------------------- API
    def reset(self, **obs_kwargs):
        """(:147-180) -- x_k carries over from the previous episode."""
        self.time_index = 0
        oob_poll(self.oob_count)
        ext, keep = self._ext(obs_kwargs)
        _lib.check(self._kernel("pgw_building_reset")(
            self.params, self._exo[0], self.num_envs, _lib.dptr(self.x), _lib.dptr(self.p_consumed),
            _lib.dptr(self._reward_state), ext, self._mat(self._obs), self._stream()))
        self._prev_viol_reward = None
        return self._obs

    def step(self, action, **obs_kwargs):
        """(:183-225).  Standalone: returns the reward of the PREVIOUS state (:215);
        inside a MultiComponentEnv the reward is the fresh one (base.py:137)."""
        a = as_action(action, self.num_envs, 6, self.device, self.dtype)
        t = self.time_index
        if t + 1 >= len(self._exo):
            raise IndexError("building stepped past the end of its exogenous data")
        ext, keep = self._ext(obs_kwargs)
        lagged = 0 if self._in_multicomponent else 1
        if self.reward_kind == "viol":
            prev = self._viol_reward()
        _lib.check(self._kernel("pgw_building_step")(
            self.params, self._exo[t], self._exo[t + 1], self.num_envs, self._mat(a),
            _lib.dptr(self.x), _lib.dptr(self.p_consumed), _lib.dptr(self._reward_out),
            _lib.dptr(self._reward_state), lagged, ext, self._mat(self._obs), self._stream()))
        self.time_index += 1
        rew = self._reward_out
        if self.reward_kind == "viol":
            rew = prev if lagged else self._viol_reward()
        return self._obs, rew, self.is_terminal(), {"p_consumed": self.p_consumed}

    @property
    def zone_temp(self):
        """[N, 5] zone temperatures (= C x_k + mean_output, dynamics.py:75-85)."""
        C = torch.tensor([self.params.C[z] for z in range(5)], dtype=torch.float64, device=self.device)
        mu = torch.tensor([self.params.mean[z] for z in range(5)], dtype=torch.float64, device=self.device)
        return (C[:, None] * self.x + mu[:, None]).t()

    def _viol_reward(self):
        """FiveZoneROMEnv.step_reward (:286-297): upper-viol^2 twice, per zone [N, 5]."""
        ub = self._cb[self.time_index, 1]
        v = self.zone_temp - ub
        return v ** 2 + v ** 2

    def get_obs(self, **obs_kwargs):
        return self._obs, {"p_consumed": self.p_consumed}

    # ---- fused MultiComponentEnv step (pgw_mc_agent_step): same as step() in an MC
    def _mc_static(self, args, slot):
        args.bld, args.bld_ext = self.params, _lib.BuildingExt()
        args.bld_x, args.bld_reward_state = self.x.data_ptr(), self._reward_state.data_ptr()
        c = args.comp[slot]
        c.kind, c.obs, c.real_power = 0, self._mat(self._obs), self.p_consumed.data_ptr()

    def _mc_prepare(self, args, slot, action, obs_kwargs):
        a, m = self._action_mat(action, 6)
        t = self.time_index
        if t + 1 >= len(self._exo):
            raise IndexError("building stepped past the end of its exogenous data")
        keep = None
        if obs_kwargs:
            args.bld_ext, keep = self._ext(obs_kwargs)
        elif args.bld_ext.bus_voltage or args.bld_ext.min_voltage or args.bld_ext.max_voltage or \
                args.bld_ext.p_setpoint:
            args.bld_ext = _lib.BuildingExt()
        args.bld_ex_t, args.bld_ex_next = self._exo[t], self._exo[t + 1]
        args.comp[slot].action = m
        return a, keep

    def _mc_dyn_k(self):
        return self.time_index

    def _mc_dyn_len(self):
        return len(self._exo) - 1

    def _mc_dyn(self, rec, k):
        rec.bld_ex_t, rec.bld_ex_next = self._exo[k], self._exo[k + 1]

    def _mc_replayed(self):
        pass

    def _mc_finish(self, obs_kwargs):
        self.time_index += 1
        return self._obs, self._reward_state, self.is_terminal(), {"p_consumed": self.p_consumed}

    def step_reward(self):
        if self.reward_kind == "viol":
            return self._viol_reward(), {}
        return self._reward_state, {}

    def _current_reward(self):
        if self.reward_kind == "viol":
            raise NotImplementedError("FiveZoneROMEnv's vector reward cannot be summed in a "
                                      "MultiComponentEnv (use FiveZoneROMThermalEnergyEnv)")
        return self._reward_state

    def is_terminal(self) -> bool:
        return self.time_index == self.max_episode_steps - 1                # :289-293

    @property
    def real_power(self):
        return self.p_consumed                                              # :305-308


@register_env
class FiveZoneROMThermalEnergyEnv(FiveZoneROMEnv):
    """Same physics, reward 0.2*0.5*(-P/12) - 0.8*sum(max(viol, 0)^2) (:312-335)."""

    fused_kind = "building"
    reward_kind = "thermal_energy"
    mc_kind = 0
