"""Debug: heterogeneous scenario at 65,536 envs vs its golden (which obs columns differ)."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.conftest import golden_path
from powergridworld_amd.multiagent_env import MultiAgentEnv
from powergridworld_amd.scenarios.heterogeneous import make_env_config
DEV = "cuda:0"
with np.load(golden_path("het_scenario"), allow_pickle=False) as z:
    g = {k: z[k] for k in z.files}
Tn, K, _ = g["actions"].shape
for n in (int(sys.argv[1]) if len(sys.argv) > 1 else 65536, 64):
    rep = n // K
    env = MultiAgentEnv(**make_env_config(), num_envs=n, device=DEV)
    env.reset()
    env.agent_dict["building"].env_dict["storage"].reset(init_storage=torch.tensor(np.tile(g["init_storage"], rep), device=DEV))
    acts = torch.tensor(np.tile(g["actions"], (1, rep, 1)), device=DEV)
    a = acts[0]
    act = {"building": {"building": a[:, :6], "pv": a[:, 6:7], "storage": a[:, 7:8]}, "pv": a[:, 8:9], "ev-charging": a[:, 9:10]}
    obs, rew, dones, _ = env.step(act)
    o = torch.cat([obs["building"]["building"], obs["building"]["pv"], obs["building"]["storage"], obs["pv"], obs["ev-charging"]], 1).cpu().numpy()
    want = np.tile(g["obs"][1], (rep, 1))
    bad = ~np.isclose(o, want, rtol=1e-9, atol=1e-9)
    print("n", n, "bad per column", bad.sum(0).tolist())
    rows = np.nonzero(bad.any(1))[0]
    print("ev got", o[:4, 19:], "\nev want", want[:4, 19:])
    print("ev rp", env.agent_dict["ev-charging"].real_power[:4].tolist(), "rew", rew["ev-charging"][:4].tolist(), "want rew", g["reward"][0])
    b20 = bad[:, 20]
    print("bad by lane", b20[: n // 64 * 64].reshape(-1, 64).sum(0).tolist())
    print("bad by block (first 16)", b20[: n // 64 * 64].reshape(-1, 64).sum(1)[:16].tolist(), "blocks bad", int((b20[: n // 64 * 64].reshape(-1, 64).sum(1) > 0).sum()))
    print("nact values got", np.unique(o[:, 20], return_counts=True))
    if len(rows):
        r = rows[0]
        print("first bad env", r, "got", o[r][bad[r]], "want", want[r][bad[r]])
