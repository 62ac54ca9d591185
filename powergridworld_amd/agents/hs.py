"""Home-Steward components, batched (reference: gridworld/agents/pv/
pv_profile_env_hs.py, energy_storage/energy_storage_env_hs.py,
vehicles/ev_charging_env_hs.py, devices/devices_env_hs.py).

They only run inside HSMultiComponentEnv (base_hs.py), which steps the whole
chain in one kernel (pgw_hs_step): each class here holds its component's
parameters, spaces and obs labels exactly as the reference builds them, and
the house hands it views of its state.  Stepping one on its own is not
supported -- the reference's components need the house's meta_state kwargs.
"""
import json
import math
import os

import numpy as np
import pandas as pd
import torch

from powergridworld_amd import spaces
from powergridworld_amd.agents.pv import load_profile
from powergridworld_amd.base import ComponentEnv, register_env
from powergridworld_amd.utils import maybe_rescale_box_space

DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")


def load_hs_data():
    with open(os.path.join(DATA_DIR, "hs_data.json")) as f:
        return json.load(f)


class _HSComponent(ComponentEnv):
    hs_kind = None

    def reset(self, **kwargs):
        raise NotImplementedError("%s resets inside HSMultiComponentEnv" % type(self).__name__)

    def step(self, action, **kwargs):
        raise NotImplementedError("%s steps inside HSMultiComponentEnv" % type(self).__name__)

    def step_reward(self, **kwargs):
        raise NotImplementedError("the house evaluates its components' rewards (base_hs.py:183-199)")

    def get_obs(self, **kwargs):
        return self._obs, {}

    def _adopt(self, obs):
        self._obs = obs


@register_env
class HSPVEnv(_HSComponent):
    """pv_profile_env_hs.py:15-98: action box (0.98, 1), obs -data[index]
    (+ min_voltage when grid_aware)."""

    hs_kind = 0

    def __init__(self, name: str = None, profile_csv: str = None, profile_path: str = None,
                 profile_data: list = [], scaling_factor: float = 1., rescale_spaces: bool = True,
                 grid_aware: bool = False, max_episode_steps: int = None, minutes_per_step: int = 5,
                 num_envs: int = 1, device=None, **kwargs):
        super().__init__(name=name, num_envs=num_envs, device=device)
        self.grid_aware = bool(grid_aware)
        self.scaling_factor = scaling_factor
        self.rescale_spaces = rescale_spaces
        self.minutes_per_step = minutes_per_step
        if len(profile_data) != 0:
            data = np.array(profile_data, dtype=np.float64)
        else:
            data = load_profile(profile_csv, profile_path)
        self.data = np.array([scaling_factor * float(i) for i in data])     # :67
        self.episode_length = len(self.data)
        if max_episode_steps is not None:
            self.episode_length = min(max_episode_steps, self.episode_length)
        # grid_aware (:47-48, 81-85): min_voltage joins the obs, box (0.9, 1.1); the
        # house takes it as a step / reset keyword (MultiAgentEnv passes it)
        self._obs_labels = ["real_power"] + (["min_voltage"] if self.grid_aware else [])
        lo, hi = [-np.max(self.data)], [0.]
        if self.grid_aware:
            lo, hi = lo + [0.9], hi + [1.1]
        self._observation_space = spaces.Box(shape=(len(lo),), low=np.array(lo), high=np.array(hi),
                                             dtype=np.float64)
        self.observation_space = maybe_rescale_box_space(self._observation_space, rescale_spaces)
        self._action_space = spaces.Box(shape=(1,), low=0.98, high=1., dtype=np.float64)
        self.action_space = maybe_rescale_box_space(self._action_space, rescale_spaces)
        self.index = None


@register_env
class HSEnergyStorageEnv(_HSComponent):
    """energy_storage_env_hs.py:10-74: SoC and the stored energy's cost."""

    hs_kind = 1

    def __init__(self, name: str = None, storage_range: tuple = (3.0, 50.0), initial_storage_mean: float = 30.0,
                 initial_storage_std: float = 5.0, charge_efficiency: float = 0.95,
                 discharge_efficiency: float = 0.9, max_power: float = 15.0, max_episode_steps: int = 288,
                 control_timedelta: pd.Timedelta = pd.Timedelta(300, "s"), rescale_spaces: bool = True,
                 initial_storage_cost: float = 0.0, max_storage_cost: float = 0.55, num_envs: int = 1,
                 device=None, **kwargs):
        super().__init__(name=name, num_envs=num_envs, device=device)
        self.initial_storage_cost = initial_storage_cost
        self.storage_range = tuple(storage_range)
        self.initial_storage_mean = initial_storage_mean
        self.initial_storage_std = initial_storage_std
        self.charge_efficiency = charge_efficiency
        self.discharge_efficiency = discharge_efficiency
        self.max_power = max_power
        self.rescale_spaces = rescale_spaces
        self.max_storage_cost = max_storage_cost
        self.max_episode_steps = max_episode_steps
        self.control_interval_in_hr = pd.Timedelta(control_timedelta).seconds / 3600.0
        self.simulation_step = 0
        self._obs_labels = ["stage_of_charge", "cost"]     # sic (:57)
        self._observation_space = spaces.Box(shape=(2,), low=np.array([self.storage_range[0], 0.00]),
                                             high=np.array([self.storage_range[1], max_storage_cost]),
                                             dtype=np.float64)
        self.observation_space = maybe_rescale_box_space(self._observation_space, rescale_spaces)
        self._action_space = spaces.Box(shape=(1,), low=-1.0, high=1.0, dtype=np.float64)
        self.action_space = maybe_rescale_box_space(self._action_space, rescale_spaces)
        n = self.num_envs
        self.soc = torch.zeros(n, dtype=torch.float64, device=self.device)
        self.cost = torch.full((n,), float(initial_storage_cost), dtype=torch.float64, device=self.device)
        self._gen = torch.Generator(device=self.device)
        self.seed(None)

    @property
    def current_storage(self):
        return self.soc

    @property
    def current_cost(self):
        return self.cost

    def initial_soc(self, init_storage=None):
        """reset's SoC (:80-105): clip(init_storage), or the truncated normal draw
        truncnorm(-1, 1) * std + mean, drawn on the device by inverse-CDF sampling
        (z = sqrt(2) erfinv(2 u' - 1), u' ~ U[Phi(-1), Phi(1)]), as
        EnergyStorageEnv does: scipy's host sampler cost ~4 ms per reset at
        65 536 envs (14 us per step of a 286-step episode)."""
        if init_storage is None:
            lo = 0.5 * (1.0 + math.erf(-1.0 / math.sqrt(2.0)))
            hi = 0.5 * (1.0 + math.erf(1.0 / math.sqrt(2.0)))
            u = torch.rand(self.num_envs, dtype=torch.float64, device=self.device, generator=self._gen)
            z = math.sqrt(2.0) * torch.special.erfinv(2.0 * (lo + u * (hi - lo)) - 1.0)
            return z * self.initial_storage_std + self.initial_storage_mean
        t = init_storage if isinstance(init_storage, torch.Tensor) else torch.as_tensor(
            np.asarray(init_storage, dtype=np.float64))
        t = t.to(device=self.device, dtype=torch.float64).reshape(-1)
        if t.numel() == 1:
            t = t.expand(self.num_envs)
        return t.contiguous()

    def seed(self, seed=None):
        """Seed the initial-SoC sampler (the reference draws from NumPy's global RNG)."""
        self._gen.manual_seed(int(seed) if seed is not None else int(torch.seed() % (2 ** 63)))


@register_env
class HSEVChargingEnv(_HSComponent):
    """ev_charging_env_hs.py:14-125: every vehicle of the table (num_vehicles
    only sizes the obs bounds), times rounded down to the step."""

    hs_kind = 2

    def __init__(self, num_vehicles: int = 100, minutes_per_step: int = 5, max_charge_rate_kw: float = 7.0,
                 max_episode_steps: int = None, unserved_penalty: float = 1., peak_penalty: float = 1.,
                 peak_threshold: float = 10., reward_scale: float = 1e5, name: str = None,
                 randomize: bool = False, vehicle_csv: str = None, vehicle_multiplier: int = 1,
                 rescale_spaces: bool = True, max_charge_cost: float = 0.55, profile_data: dict = {},
                 num_envs: int = 1, device=None, **kwargs):
        super().__init__(name=name, num_envs=num_envs, device=device)
        self.num_vehicles = num_vehicles
        self.max_charge_rate_kw = max_charge_rate_kw
        self.minutes_per_step = minutes_per_step
        self.vehicle_multiplier = vehicle_multiplier
        self.rescale_spaces = rescale_spaces
        self.unserved_penalty = unserved_penalty
        self.max_episode_steps = max_episode_steps if max_episode_steps is not None else np.inf
        self.max_episode_steps = min(self.max_episode_steps, 24 * 60 / minutes_per_step)
        self.simulation_times = np.arange(0, (self.max_episode_steps + 1) * minutes_per_step, minutes_per_step)
        if profile_data != {}:
            split = profile_data
        elif vehicle_csv:
            split = json.loads(pd.read_csv(vehicle_csv).to_json(orient="split"))
        else:
            split = load_hs_data()["vehicles_hs"]
        df = pd.DataFrame(split["data"], columns=split["columns"])
        req = df["energy_required_kwh"].to_numpy(np.float64) * self.vehicle_multiplier
        rnd = lambda x: x - x % self.minutes_per_step                              # :247
        self.start_min = rnd(df["start_time_min"].to_numpy(np.float64))
        self.end_park_min = rnd(df["end_time_park_min"].to_numpy(np.float64))
        self.req0 = req
        if len(req) > 64:
            raise ValueError("at most 64 vehicles per HS house")
        bounds = [(0, self.simulation_times[-1]), (0, num_vehicles), (0, num_vehicles * max_charge_rate_kw),
                  (0, num_vehicles * req.max()), (0, req.max() / (minutes_per_step / 60.)),
                  (0, req.max()), (0, max_charge_cost)]
        self.obs_low = np.array([b[0] for b in bounds], dtype=np.float64)
        self.obs_high = np.array([b[1] for b in bounds], dtype=np.float64)
        self._observation_space = spaces.Box(low=self.obs_low, high=self.obs_high, shape=(7,), dtype=np.float64)
        self.observation_space = maybe_rescale_box_space(self._observation_space, rescale_spaces)
        self._action_space = spaces.Box(low=0., high=1., shape=(1,), dtype=np.float64)
        self.action_space = maybe_rescale_box_space(self._action_space, rescale_spaces)
        self._obs_labels = ["time", "num_active_vehicles", "real_power_consumed", "real_power_demand",
                            "mean_charge_rate_deficit", "real_power_unserved", "current_cost"]
        self.time_index = None
        self.time = None

    def window(self, time):
        """Bit v: vehicle v parked at `time` (:208-210)."""
        bits = 0
        for v in range(len(self.req0)):
            if time >= np.floor(self.start_min[v]) and time <= np.floor(self.end_park_min[v]):
                bits |= 1 << v
        return bits


@register_env
class HSDevicesEnv(_HSComponent):
    """devices_env_hs.py:13-104: other household loads from a profile."""

    hs_kind = 3

    def __init__(self, name: str = None, profile_csv: str = None, profile_path: str = None,
                 profile_data: dict = {}, scaling_factor: float = 1., rescale_spaces: bool = True,
                 max_episode_steps: int = None, minutes_per_step: int = 5, num_envs: int = 1, device=None,
                 **kwargs):
        super().__init__(name=name, num_envs=num_envs, device=device)
        self.scaling_factor = scaling_factor
        self.rescale_spaces = rescale_spaces
        self.minutes_per_step = minutes_per_step
        if profile_data != {}:
            self.data_pd = pd.DataFrame(np.array([v for v in profile_data.values()]).T,
                                        columns=list(profile_data.keys()))
        elif profile_path is not None:
            self.data_pd = pd.read_csv(profile_path)
        else:
            d = load_hs_data()["devices_profile_hs"]
            self.data_pd = pd.DataFrame({k: np.asarray(v, dtype=np.float64) for k, v in d.items()})
        self.data = self.data_pd.values[0:, :].squeeze() * self.scaling_factor
        self.episode_length = len(self.data)
        if max_episode_steps is not None:
            self.episode_length = min(max_episode_steps, self.episode_length)
        self._obs_labels = list(self.data_pd.columns)
        if len(self._obs_labels) > 4:
            raise ValueError("at most 4 device profiles")
        self.obs_high = np.array([max(list(self.data_pd[c])) for c in self._obs_labels], dtype=np.float64)
        self._observation_space = spaces.Box(shape=(len(self._obs_labels),),
                                             low=np.zeros(len(self._obs_labels)), high=self.obs_high,
                                             dtype=np.float64)
        self.observation_space = maybe_rescale_box_space(self._observation_space, rescale_spaces)
        self._action_space = spaces.Box(shape=(1,), low=0.99, high=1., dtype=np.float64)
        self.action_space = maybe_rescale_box_space(self._action_space, rescale_spaces)
        self.index = None
