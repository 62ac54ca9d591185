"""Batched HSMultiComponentEnv (reference: gridworld/base_hs.py:12-199).

The Home-Steward house: PV, battery, EV charger and other devices share the
PV / battery / grid power of each 5-minute step in a fixed order -- each
component draws on what the previous ones left and the weighted cost of what
it drew feeds its reward.  The reference passes that state down the chain in a
`meta_state` dict; here the whole chain runs in one kernel per step
(pgw_hs_step, one thread per env, include/pgw.h), so a step is one launch
whatever the number of envs.

Differences from the reference, all of them batching:
  * obs / reward / real_power are [N] / [N, dim] fp64 device tensors (views of
    the house's buffers: copy them to keep them across steps);
  * the returned meta is the batched meta_state: timestamp and grid_cost
    (shared), pv_power / es_power / grid_power ([N]); the per-device
    `step_meta` logging records are not produced;
  * reset(init_storage=...) accepts a per-env [N] SoC.
"""
from typing import List

import numpy as np
import pandas as pd
import torch

from powergridworld_amd import _lib
from powergridworld_amd.base import MultiComponentEnv, as_action, as_env_tensor, oob_poll, register_env


# device_custom_info keys of each HS kind's step_meta record, in the reference's
# order (PGW_HS_META_FIELDS, include/pgw.h): fields 6.. of the record
HS_CUSTOM_INFO = {
    0: ("pv_available_power", "pv_actionable_power"),                         # pv_profile_env_hs.py:155
    1: ("current_storage", "power_ask", "solar_power_available", "grid_power_available",
        "es_power_available"),                                                # energy_storage_env_hs.py:261
    2: ("power_ask", "power_unserved", "charging_vehicle", "vehicle_charged", "solar_power_available",
        "es_power_available", "grid_power_available"),                        # ev_charging_env_hs.py:320
    3: ("power_ask", "solar_power_available", "es_power_available", "grid_power_available"),  # devices :199
}
HS_META_FIELDS = 13
HS_COMMON_FIELDS = ("cost", "reward", "action", "solar_power_consumed", "es_power_consumed",
                    "grid_power_consumed")


@register_env
class HSMultiComponentEnv(MultiComponentEnv):
    """step_meta=True (default, as the reference): meta["step_meta"] is the
    per-device record list base_hs.py:133-164 builds, one dict per chain slot
    with the reference's keys; every numeric entry is an [N] device tensor (a
    view of the kernel's record buffer, overwritten by the next step; `action`
    is the raw action, where the reference holds a one-element list)."""

    def __init__(self, name: str = None, components: List[dict] = None, start_time: str = "",
                 end_time: str = "", control_timedelta=pd.Timedelta(300, "s"), max_grid_power: float = 48,
                 max_episode_steps: int = None, rescale_spaces: bool = True, num_envs: int = 1,
                 device=None, step_meta: bool = True, **kwargs):
        self.max_grid_power = max_grid_power
        self._want_step_meta = bool(step_meta)
        super().__init__(name=name, components=components, num_envs=num_envs, device=device)
        from powergridworld_amd.agents.hs import _HSComponent
        self.rescale_spaces = rescale_spaces
        self._grid_cost_data = [float(x) for x in kwargs["grid_cost"]]
        self._timestamps = kwargs["timestamps"]
        self.max_episode_steps = max_episode_steps if max_episode_steps is not None else np.inf
        kinds = []
        for e in self.envs:
            if not isinstance(e, _HSComponent):
                raise TypeError("HSMultiComponentEnv components must be HS components, got %s"
                                % type(e).__name__)
            kinds.append(e.hs_kind)
        if len(set(kinds)) != len(kinds):
            raise ValueError("each HS component kind may appear once")
        if kinds[0] != 0:
            # meta_state pv_power is None until the PV's first step (base_hs.py:58):
            # in the reference a component ahead of the PV raises TypeError in its
            # first reset / step (the EV's reset step and every step_meta subtract
            # from it); the order after the PV is free
            raise NotImplementedError("the HS chain must start with the PV (it sets pv_power)")
        self._kinds = kinds
        self._by_kind = {k: e for k, e in zip(kinds, self.envs)}
        self.time_index = None
        self.meta_state = {"timestamp": None, "grid_cost": None, "es_cost": 0.0, "grid_power": None,
                           "pv_power": None, "es_power": None, "pv_cost": 0.0}
        self._setup()

    # ------------------------------------------------------------ buffers, params
    def _setup(self):
        n, dev = self.num_envs, self.device
        p = _lib.HSParams()
        p.n_comp = len(self.envs)
        off = 0
        dims = []
        for c, (k, e) in enumerate(zip(self._kinds, self.envs)):
            p.kind[c] = k
            p.obs_off[c] = off
            p.rescale[c] = int(bool(e.rescale_spaces))
            d = e._observation_space.shape[0]
            dims.append(d)
            off += d
        self._obs_dim = off
        pv = self._by_kind.get(0)
        if pv is not None:
            p.pv_act_low, p.pv_act_high = 0.98, 1.0
            p.pv_obs_low = float(-np.max(pv.data))
        st = self._by_kind.get(1)
        if st is not None:
            p.soc_min, p.soc_max = float(st.storage_range[0]), float(st.storage_range[1])
            if max(st.storage_range) != p.soc_max:
                raise ValueError("storage_range must be (low, high)")
            p.eta_c, p.eta_d = float(st.charge_efficiency), float(st.discharge_efficiency)
            p.max_power, p.dt_h = float(st.max_power), float(st.control_interval_in_hr)
            p.max_storage_cost = float(st.max_storage_cost)
        ev = self._by_kind.get(2)
        if ev is not None:
            p.n_veh = len(ev.req0)
            p.ev_rate = float(ev.max_charge_rate_kw)
            p.ev_hours_per_step = ev.minutes_per_step / 60.
            p.ev_steps_per_hour = 60.0 / ev.minutes_per_step
            p.ev_mult = float(ev.vehicle_multiplier)
            p.ev_unserved_penalty = float(ev.unserved_penalty)
            for j in range(7):
                p.ev_obs_low[j], p.ev_obs_high[j] = ev.obs_low[j], ev.obs_high[j]
            for v in range(p.n_veh):
                p.ev_end_park[v] = ev.end_park_min[v]
                p.ev_req0[v] = ev.req0[v]
        dv = self._by_kind.get(3)
        if dv is not None:
            p.n_dev = len(dv._obs_labels)
            p.dev_act_low, p.dev_act_high = 0.99, 1.0
            p.dev_hours_per_step = dv.minutes_per_step / 60.0
            for j in range(p.n_dev):
                p.dev_obs_high[j] = dv.obs_high[j]
        p.max_grid_power = float(self.max_grid_power)
        p.pv_grid_aware = int(bool(pv is not None and pv.grid_aware))
        self.params = p
        self._bind_oob(self.oob_count)

        f64 = dict(dtype=torch.float64, device=dev)
        self._obs_buf = torch.zeros((self._obs_dim, n), **f64)
        self._act_buf = torch.zeros((len(self.envs), n), **f64)
        for c, e in enumerate(self.envs):
            e._adopt(self._obs_buf[p.obs_off[c]:p.obs_off[c] + dims[c]].t())
        st_soc = st.soc if st is not None else torch.zeros(n, **f64)
        st_cost = st.cost if st is not None else torch.zeros(n, **f64)
        self._ev_req = torch.zeros((max(p.n_veh, 1), n), **f64)
        self._ev_chg = torch.zeros(n, dtype=torch.int64, device=dev)
        self._ev_cost = torch.zeros(n, **f64)
        self._dev_cost = torch.zeros(n, **f64)
        self._es_last = torch.zeros(n, **f64)       # meta_state es_power = 0.0 (base_hs.py:59)
        # meta_state pv_power (base_hs.py:58: None until the PV's first step; NaN here):
        # carried from step to step, so components ahead of the PV see the last one
        self._pv_last = torch.full((n,), float("nan"), **f64)
        self._mv_state = None          # meta_state min_voltage (set by the first step)
        self._reward = torch.zeros(n, **f64)
        self._meta = torch.zeros((3, n), **f64)
        self._init_soc = torch.zeros(n, **f64)
        b = _lib.HSBuffers()
        b.action = _lib.Mat(self._act_buf.data_ptr(), 1, n)
        b.obs = _lib.Mat(self._obs_buf.data_ptr(), 1, n)
        b.soc, b.soc_cost = st_soc.data_ptr(), st_cost.data_ptr()
        b.ev_req, b.ev_charging = self._ev_req.data_ptr(), self._ev_chg.data_ptr()
        b.ev_cost, b.dev_cost = self._ev_cost.data_ptr(), self._dev_cost.data_ptr()
        b.es_power_last = self._es_last.data_ptr()
        b.pv_power_last = self._pv_last.data_ptr()
        b.reward, b.real_power = self._reward.data_ptr(), self._real_power.data_ptr()
        b.meta_out = self._meta.data_ptr()
        self._step_meta = None
        if self._want_step_meta:
            self._rec_buf = torch.zeros((len(self.envs), HS_META_FIELDS, n), **f64)
            b.step_meta = self._rec_buf.data_ptr()
            self._step_meta = []
            for c, (k, e) in enumerate(zip(self._kinds, self.envs)):
                r = {"device_id": e.name, "timestamp": None}
                r.update({f: self._rec_buf[c, j] for j, f in enumerate(HS_COMMON_FIELDS)})
                r["device_custom_info"] = {f: self._rec_buf[c, 6 + j] for j, f in enumerate(HS_CUSTOM_INFO[k])}
                self._step_meta.append(r)
        self._bufs = b
        self._keep = (st_soc, st_cost)
        self._act_key = None
        self._info_cache = {}
        if dv is not None:
            self._dev_power = self._dev_rows(dv)

    @staticmethod
    def _dev_rows(dv):
        return np.stack([dv.data_pd[c].to_numpy(np.float64) for c in dv._obs_labels], 1)

    def _info(self, ev_time, ev_next_time):
        """Shared per-step values: data rows of PV / devices, grid cost, EV times
        (cached per (row indices, time): every env shares them)."""
        pv, dv = self._by_kind.get(0), self._by_kind.get(3)
        key = (pv.index if pv is not None else -1, dv.index if dv is not None else -1, self.time_index,
               ev_time, ev_next_time)
        s = self._info_cache.get(key)
        if s is None:
            if len(self._info_cache) > 4096:
                self._info_cache.clear()
            s = self._info_cache[key] = self._make_info(ev_time, ev_next_time)
        return s

    def _make_info(self, ev_time, ev_next_time, rows=None):
        """`rows` = (PV row, devices row, house time index); None: the present ones."""
        s = _lib.HSStepInfo()
        pv, dv = self._by_kind.get(0), self._by_kind.get(3)
        pi, di, ti = rows if rows is not None else (pv.index if pv is not None else 0,
                                                    dv.index if dv is not None else 0, self.time_index)
        if pv is not None:
            s.pv_avail = float(pv.data[pi])
        s.grid_cost = self._grid_cost_data[ti]
        if dv is not None:
            for j, c in enumerate(dv._obs_labels):
                s.dev_obs[j] = float(dv.data[di][j]) if np.ndim(dv.data) > 1 else float(dv.data[di])
                s.dev_power[j] = float(self._dev_power[di, j])
        ev = self._by_kind.get(2)
        if ev is not None:
            s.ev_time, s.ev_next_time = float(ev_time), float(ev_next_time)
            s.ev_window = ev.window(ev_time)
        return s

    # ------------------------------------------------------------ API
    def reset(self, **kwargs):
        """base_hs.py:66-91: every component to row 0, the EV's action-less step."""
        self.time_index = 0
        oob_poll(self.oob_count)
        self.meta_state["timestamp"] = self._timestamps[self.time_index]
        self.meta_state["grid_cost"] = self._grid_cost_data[self.time_index]
        self.meta_state["grid_power"] = self.max_grid_power
        for k, e in self._by_kind.items():
            if k in (0, 3):
                e.index = 0
        st = self._by_kind.get(1)
        if st is not None:
            st.simulation_step = 0
            soc0 = st.initial_soc(kwargs.get("init_storage"))
        else:
            soc0 = torch.zeros(self.num_envs, dtype=torch.float64, device=self.device)
        self._init_soc.copy_(soc0)
        ev = self._by_kind.get(2)
        t0 = 0.0
        if ev is not None:
            ev.time_index = 0
            ev.time = t0 = ev.simulation_times[0]
        s = self._info(t0, t0)
        self._bind_min_voltage(kwargs)
        _lib.check(_lib.lib().pgw_hs_reset(self.params, s, self.num_envs, _lib.dptr(self._init_soc),
                                           self._bufs, self._stream()))
        if ev is not None:
            ev.time = ev.simulation_times[ev.time_index]
            ev.time_index += 1
        return self.get_obs(**kwargs)[0]

    def _bind_min_voltage(self, kwargs, stepping=False):
        """The grid-aware PV's min_voltage (pv_profile_env_hs.py:110-111 reads
        kwargs["min_voltage"]), as the reference's house delivers it: the PV
        gets the step's keywords UPDATED WITH meta_state (base_hs.py:130-132),
        and its returned meta -- the keywords it saw, min_voltage included --
        is merged into meta_state (:147-153).  So the first step's min_voltage
        stays in meta_state and every later reset and step observes that value,
        whatever is passed then; before the first step the keyword is used.
        (Pinned by the reference's own run, tests/golden/hs_order.npz.)"""
        if not self.params.pv_grid_aware:
            return
        mv = self._mv_state
        if mv is None:
            if "min_voltage" not in kwargs:
                raise KeyError("min_voltage (the grid-aware HSPVEnv observes it)")
            mv = as_env_tensor(kwargs["min_voltage"], self.num_envs, self.device, "min_voltage").clone()
            if stepping:
                self._mv_state = mv
        self._mv_hold = mv
        self._bufs.min_voltage = mv.data_ptr()

    def get_obs(self, **kwargs):
        return {e.name: e._obs for e in self.envs}, {}

    def _pack(self, action):
        """A packed [N, n_comp] tensor is read in place (any strides); a
        {component: [N, 1]} dict is gathered into the house's action buffer."""
        if isinstance(action, torch.Tensor):
            if tuple(action.shape) != (self.num_envs, len(self.envs)):
                raise ValueError("packed HS action must be [N, %d]" % len(self.envs))
            if action.dtype != torch.float64 or action.device != self.device:
                action = action.to(device=self.device, dtype=torch.float64)
            key = (action.data_ptr(), action.stride(0), action.stride(1))
            self._act_hold = action
        else:
            for c, e in enumerate(self.envs):
                self._act_buf[c].copy_(as_action(action[e.name], self.num_envs, 1, self.device)[:, 0])
            key = (self._act_buf.data_ptr(), 1, self.num_envs)
        if key != self._act_key:                  # (Mats cached per buffer: callers cycle a few)
            mats = self.__dict__.setdefault("_act_mats", {})
            m = mats.get(key)
            if m is None:
                if len(mats) >= 64:
                    mats.clear()
                m = mats[key] = _lib.Mat(*key)
            self._bufs.action = m
            self._act_key = key

    def step(self, action, **kwargs):
        """base_hs.py:114-180.  `action`: {component: [N, 1]} or one packed [N, n_comp]."""
        self._pack(action)
        ev_time, ev_next = self._pre_step()
        s = self._info(ev_time, ev_next)
        self._bind_min_voltage(kwargs, stepping=True)
        _lib.check(_lib.lib().pgw_hs_step(self.params, s, self.num_envs, self._bufs, self._stream()))
        return self._post_step(ev_next)

    def _pre_step(self):
        """The step's host bookkeeping before the launch; (EV time, next time)."""
        self.meta_state["timestamp"] = self._timestamps[self.time_index]
        self.meta_state["grid_cost"] = self._grid_cost_data[self.time_index]
        self.meta_state["grid_power"] = self.max_grid_power
        ev = self._by_kind.get(2)
        if ev is None:
            return 0.0, 0.0
        return ev.time, ev.simulation_times[ev.time_index]

    # ---- captured steps (graph.py): step j after a reset runs at PV / devices
    # row j, house time index j and EV times (simulation_times[j], [j + 1])
    def _hs_step_k(self):
        return self.time_index

    def _hs_steps(self):
        """How many steps after a reset have data (the tables' length)."""
        lens = [len(self._grid_cost_data)]
        for k, e in self._by_kind.items():
            if k in (0, 3):
                lens.append(len(e.data))
            elif k == 2:
                lens.append(len(e.simulation_times) - 1)
        return min(lens)

    def _info_at(self, j):
        ev = self._by_kind.get(2)
        t0 = t1 = 0.0
        if ev is not None:
            t0, t1 = float(ev.simulation_times[j]), float(ev.simulation_times[j + 1])
        return self._make_info(t0, t1, rows=(j, j, j))

    def capture_step(self, action, steps=1, **kwargs):
        """A StepGraph (graph.py) of `steps` house steps reading `action` (a
        packed [N, n_comp] fp64 device tensor, or a list of `steps` of them),
        captured once per episode position on first use."""
        from powergridworld_amd.graph import StepGraph
        return StepGraph(self, action, steps, kwargs)

    def _post_step(self, ev_next):
        """The step's host bookkeeping after the launch (clocks, done, meta)."""
        dones = []
        for k, e in zip(self._kinds, self.envs):
            if k == 0:
                e.index += 1
                dones.append(e.index == e.episode_length)
            elif k == 1:
                e.simulation_step += 1
                dones.append(e.simulation_step == e.max_episode_steps)
            elif k == 2:
                dones.append(e.time_index == e.max_episode_steps)
                e.time = ev_next
                e.time_index += 1
            else:
                e.index += 1
                dones.append(e.index == e.episode_length)
        self.time_index += 1
        meta = dict(self.meta_state)
        meta.update(pv_power=self._meta[0], es_power=self._meta[1], grid_power=self._meta[2],
                    es_cost=0)
        if self._step_meta is not None:
            for r in self._step_meta:
                r["timestamp"] = meta["timestamp"]
            meta["step_meta"] = self._step_meta
        obs = {e.name: e._obs for e in self.envs}
        return obs, self._reward, any(dones), meta

    def step_reward(self, **kwargs):
        return self._reward, {}

    def _current_reward(self):
        return self._reward
