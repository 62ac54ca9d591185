"""PowerFlowSolver plugin ABC (reference: gridworld/distribution_system/powerflow.py:7-51)."""
from abc import ABC, abstractmethod
from typing import Dict


class PowerFlowSolver(ABC):
    """API of the power flow solver called from MultiAgentEnv.  Batched
    implementations take/return one value per env (tensors [N])."""

    def __init__(self, config: dict = None, **kwargs):
        return

    @abstractmethod
    def calculate_power_flow(self, p_controllable_consumed: Dict[str, any] = None,
                             q_controllable_consumed: Dict[str, any] = None, **kwargs) -> any:
        """Compute the power flow solution using p/q consumed at each bus."""
        raise NotImplementedError

    @abstractmethod
    def get_bus_voltages(self) -> Dict[str, any]:
        """Return a dict of (bus node, voltage)."""
        raise NotImplementedError

    @abstractmethod
    def get_bus_voltage_by_name(self, name: str) -> any:
        """Return the voltage for a specific bus."""
        raise NotImplementedError
