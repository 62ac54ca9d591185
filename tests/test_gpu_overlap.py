"""MultiAgentEnv(overlap_pf=True): the C4 step's power flow on a second stream
beside the next step's agents' kernel (pgw_coord_step_overlap, two alternating
buffer sets, reads joined through the returned mappings / the solver).  Every
value read through the public API equals the synchronous fused step's bit for
bit -- rewards, violation, V675.3, iteration counts, observations -- over
steps, a mid-episode reset and a state_dict round trip.  Needs an MI355X."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _pair(conv, n):
    from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config
    envs = [CoordinatedMultiBuildingControlEnv(**make_c4_config(pf_convergence=conv), num_envs=n, device=DEV,
                                               fused=True, overlap_pf=ov) for ov in (False, True)]
    assert envs[1]._fused["overlap"] is not None and envs[0]._fused.get("overlap") is None
    return envs


@pytest.mark.parametrize("conv", ["opendss", "exact"])
def test_overlap_equals_synchronous_step(conv):
    n, steps = 4096, 40
    sync, ov = _pair(conv, n)
    rng = np.random.default_rng(5)
    init = torch.tensor(rng.uniform(5.0, 45.0, size=(5, n)), device=DEV)
    acts = torch.tensor(rng.uniform(-1, 1, size=(steps, 5, n, 8)), device=DEV)
    def start(env):
        env.reset()
        for ai, agent in enumerate(env.agents):
            agent.env_dict["storage"].reset(init_storage=init[ai])
        env.load_component_state()
    for env in (sync, ov):
        start(env)
    for t in range(steps):
        if t == 25:                                  # a reset in the middle of the stream
            for env in (sync, ov):
                start(env)
        out = []
        for env in (sync, ov):
            obs, rew, done, meta = env.step(acts[t])
            out.append((env.packed_obs().clone(), torch.stack([rew[a.name] for a in env.agents]).clone(),
                        meta["voltage_violation"].clone(), env.pf_solver.get_bus_voltage_by_name("675c").clone(),
                        env.pf_solver.iterations.clone(), done["__all__"]))
        for a, b in zip(out[0][:5], out[1][:5]):
            assert torch.equal(a, b), t
        assert out[0][5] == out[1][5]
    # the state after the stream (device copies), and stepping on from a restore
    sd = ov.state_dict()
    ov2 = _pair(conv, n)[1]
    ov2.reset()
    ov2.load_state_dict(sd)
    _, r1, _, _ = ov.step(acts[0])
    _, r2, _, _ = ov2.step(acts[0])
    for a in ov.agents:
        assert torch.equal(r1[a.name], r2[a.name])
