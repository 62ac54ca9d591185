import sys, os, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from powergridworld_amd.agents import EnergyStorageEnv
env = EnergyStorageEnv(num_envs=1024, device="cuda:0")
env.reset()
a = torch.zeros((1024, 1), dtype=torch.float64, device="cuda:0")
G = env.capture_step(a, steps=4)     # alive at exit
G()
torch.cuda.synchronize()
print("ok, exiting with a live graph")
