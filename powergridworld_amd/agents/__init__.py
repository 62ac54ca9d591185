from powergridworld_amd.agents.energy_storage import EnergyStorageEnv
from powergridworld_amd.agents.pv import PVEnv
from powergridworld_amd.agents.buildings import FiveZoneROMEnv, FiveZoneROMThermalEnergyEnv
from powergridworld_amd.agents.vehicles import EVChargingEnv

__all__ = ["EnergyStorageEnv", "PVEnv", "FiveZoneROMEnv", "FiveZoneROMThermalEnergyEnv",
           "EVChargingEnv"]
