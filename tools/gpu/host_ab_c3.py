"""A/B of the C3 eager step on one box: MultiComponentEnv's fast fused path
(_mc_step_fast: arguments built once, per-step values from the device table)
against the argument-writing path (_mc_fast = False), alternating, at a
host-bound batch (256 envs) and at C3's 16 384."""
import os
import sys
import time

import torch

ROOT = os.environ.get("GRAFT_REPO_ROOT", ".")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench_configs import c3_env  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
for n in (256, 16384):
    envs = {}
    for mode in ("fast", "args"):
        env, acts = c3_env(dev, n, 16)
        env._mc_fast = mode == "fast"
        envs[mode] = (env, acts)

    def run(env, acts, k):
        env.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(k):
            _, _, d, _ = env.step(acts[i % 16])
            if d:
                env.reset()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e6

    for env, acts in envs.values():
        run(env, acts, 100)
    res = {m: [] for m in envs}
    for r in range(4):
        for m, (env, acts) in envs.items():
            res[m].append(run(env, acts, 572))
    print("n=%d " % n + "  ".join("%s %s us/step" % (m, " ".join("%.1f" % x for x in v)) for m, v in res.items()),
          flush=True)
