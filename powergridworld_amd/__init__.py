"""powergridworld_amd -- MI355X-native batched step engine with the
PowerGridworld (lmchion/PowerGridworld) env API.  See DESIGN.md."""
__version__ = "0.1.0"

from powergridworld_amd.base import ComponentEnv, MultiComponentEnv
from powergridworld_amd.multiagent_env import MultiAgentEnv
from powergridworld_amd.multiagent_list_interface_env import MultiAgentListInterfaceEnv
