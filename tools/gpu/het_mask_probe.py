import os, sys, time, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from powergridworld_amd.multiagent_env import MultiAgentEnv
from powergridworld_amd.scenarios.heterogeneous import make_env_config
dev = torch.device("cuda", 0); n = 65536
env = MultiAgentEnv(**make_env_config(), num_envs=n, device=dev)
s = env.pf_solver
calls = [0]
orig = s._od_row_mask
def wrapped(idx):
    key = (idx, s._cfg_version)
    if key not in s._od_rowmask:
        calls[0] += 1
    return orig(idx)
s._od_row_mask = wrapped
gen = torch.Generator(dev).manual_seed(0)
acts = [{ag.name: ({c.name: torch.empty((n, c.action_space.shape[0]), dtype=torch.float64, device=dev).uniform_(-1, 1, generator=gen) for c in ag.envs} if hasattr(ag, "envs") else torch.empty((n, ag.action_space.shape[0]), dtype=torch.float64, device=dev).uniform_(-1, 1, generator=gen)) for ag in env.agents} for _ in range(8)]
env.reset(); k = 0
for ep in range(3):
    c0, v0 = calls[0], s._cfg_version
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for t in range(286):
        _, _, d, _ = env.step(acts[k % 8]); k += 1
        if d["__all__"]:
            env.reset()
    torch.cuda.synchronize()
    print("episode", ep, "us/step %.2f" % ((time.perf_counter() - t0) / 286 * 1e6), "lazy mask computations", calls[0] - c0,
          "cfg_version", v0, "->", s._cfg_version, "masks cached", len(s._od_rowmask), flush=True)
