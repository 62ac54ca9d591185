"""The reference's 3-agent heterogeneous scenario, batched
(gridworld/scenarios/heterogeneous.py:13-112): a MultiComponentEnv building
(building + PV + storage), a grid-aware PV farm rewarded for keeping the
feeder's minimum voltage inside [0.95, 1.05], and 25 EVs x 40, all on load
675c of the IEEE-13 feeder.  The PV farm observes min_voltage (the minimum over
all node voltages of the previous power flow, multiagent_env.py:107-113) and
is rewarded on it.  By default MultiAgentEnv runs it on the fused multi-agent
path (pgw_ma_step: every agent in one launch plus the power flow); fused=False
selects the generic path (per-agent kernels, the reward as a Python hook on
[N] tensors)."""
import pandas as pd
import torch

from powergridworld_amd import _lib
from powergridworld_amd.base import as_env_tensor
from powergridworld_amd.agents.energy_storage import EnergyStorageEnv
from powergridworld_amd.agents.buildings import FiveZoneROMThermalEnergyEnv
from powergridworld_amd.agents.pv import PVEnv
from powergridworld_amd.agents.vehicles import EVChargingEnv
from powergridworld_amd.base import MultiComponentEnv, register_env
from powergridworld_amd.distribution_system.opendss import OpenDSSSolver


@register_env
class ThisPVEnv(PVEnv):
    """PV farm rewarded on the bus voltage (heterogeneous.py:47-54):
    -(1000 (min(0, v - 0.95) + min(0, 1.05 - v)))^2 with v = min_voltage.
    The fused multi-agent step (pgw_ma_step) evaluates the same expression in its
    kernel when this class declares it here: (lo, hi, scale)."""

    fused_band_reward = (0.95, 1.05, 1000.0)

    def _band_buffer(self):
        if self.__dict__.get("_band_rew") is None:
            self._band_rew = torch.empty(self.num_envs, dtype=torch.float64, device=self.device)
        return self._band_rew

    def step_reward(self, **kwargs):
        v = as_env_tensor(kwargs["min_voltage"], self.num_envs, self.device, "min_voltage")
        self._band_buffer()
        lo, hi, scale = self.fused_band_reward
        # one kernel: -(1000 (min(0, v - 0.95) + min(0, 1.05 - v)))^2
        _lib.check(_lib.lib().pgw_voltage_band_penalty(self.num_envs, v.data_ptr(), lo, hi, scale,
                                                        self._band_rew.data_ptr(), self._stream()))
        return self._band_rew, {}


def make_env_config(system_load_rescale_factor=0.65, rescale_spaces=True, pf_convergence="opendss"):
    """heterogeneous.py:13-112 (the building's reward_structure kwarg is passed
    on unchanged; the reference's FiveZoneROMThermalEnergyEnv ignores it)."""
    building_components = [
        {"name": "building", "cls": FiveZoneROMThermalEnergyEnv,
         "config": {"reward_structure": {"alpha": 0.0}, "rescale_spaces": rescale_spaces}},
        {"name": "pv", "cls": PVEnv,
         "config": {"profile_csv": "off-peak.csv", "scaling_factor": 40., "rescale_spaces": rescale_spaces}},
        {"name": "storage", "cls": EnergyStorageEnv,
         "config": {"max_power": 20., "storage_range": (3., 250.), "rescale_spaces": rescale_spaces}},
    ]
    common_config = {
        "start_time": "08-12-2020 00:00:00",
        "end_time": "08-13-2020 00:00:00",
        "control_timedelta": pd.Timedelta(300, "s"),
    }
    pf_config = {
        "cls": OpenDSSSolver,
        "config": {
            "feeder_file": "ieee_13_dss/IEEE13Nodeckt.dss",
            "loadshape_file": "ieee_13_dss/annual_hourly_load_profile.csv",
            "system_load_rescale_factor": system_load_rescale_factor,
        },
    }
    # OpenDSSSolver(convergence=...): "opendss" = OpenDSS's snap iterate (the
    # reference's rule, the default), "exact" = the fixed point (opt-in)
    pf_config["config"]["convergence"] = pf_convergence
    agents = [
        {"name": "building", "bus": "675c", "cls": MultiComponentEnv,
         "config": {"components": building_components}},
        {"name": "pv", "bus": "675c", "cls": ThisPVEnv,
         "config": {"profile_csv": "constant.csv", "scaling_factor": 400.,
                    "rescale_spaces": rescale_spaces, "grid_aware": True}},
        {"name": "ev-charging", "bus": "675c", "cls": EVChargingEnv,
         "config": {"num_vehicles": 25, "minutes_per_step": 5, "max_charge_rate_kw": 7.,
                    "peak_threshold": 200., "vehicle_multiplier": 40., "rescale_spaces": rescale_spaces}},
    ]
    return {"common_config": common_config, "pf_config": pf_config, "agents": agents}
