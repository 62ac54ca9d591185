"""RLlib-shaped adapter (powergridworld_amd/vector_env.py):
per-sub-env structures are views of the batched engine's tensors, and
stepping through the adapter equals stepping the batch directly.  Needs an
MI355X."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _pair(n, fused):
    from powergridworld_amd.scenarios.coordinated import CoordinatedMultiBuildingControlEnv, make_c4_config
    envs = []
    for _ in range(2):
        env = CoordinatedMultiBuildingControlEnv(**make_c4_config(), num_envs=n, device=DEV, fused=fused)
        for k, agent in enumerate(env.agents):
            agent.env_dict["storage"].seed(100 + k)
        envs.append(env)
    return envs


def _batched_actions(env, rng, n):
    return {a.name: {"building": torch.tensor(rng.uniform(-1, 1, (n, 6)), device=DEV),
                     "pv": torch.tensor(rng.uniform(-1, 1, (n, 1)), device=DEV),
                     "storage": torch.tensor(rng.uniform(-1, 1, (n, 1)), device=DEV)} for a in env.agents}


def _split(act, n):
    return [{a: {c: v[i] for c, v in comps.items()} for a, comps in act.items()} for i in range(n)]


def _eq(x, y):
    if isinstance(x, dict):
        assert x.keys() == y.keys()
        for k in x:
            _eq(x[k], y[k])
    elif isinstance(x, torch.Tensor):
        assert torch.equal(x, y)
    else:
        assert x == y


@pytest.mark.parametrize("fused", [True, False])
def test_vector_env_equals_batch(fused):
    from powergridworld_amd.vector_env import MultiAgentVectorEnv
    n = 6
    ref, env = _pair(n, fused)
    venv = MultiAgentVectorEnv(env)
    obs_ref = ref.reset()
    obs = venv.vector_reset()
    assert len(obs) == n
    for i in range(n):
        _eq(obs[i], {a: {c: v[i] for c, v in comps.items()} for a, comps in obs_ref.items()})
    _eq(venv.reset_at(1), obs[1])                # still the reset's boundary: no new reset
    rng = np.random.default_rng(5)
    for t in range(5):
        act = _batched_actions(ref, rng, n)
        o_r, r_r, d_r, m_r = ref.step(act)
        o, r, d, m = venv.vector_step(_split(act, n))
        for i in range(n):
            _eq(o[i], {a: {c: v[i] for c, v in comps.items()} for a, comps in o_r.items()})
            _eq(r[i], {a: v[i] for a, v in r_r.items()})
            assert d[i] == d_r
            assert torch.equal(m[i]["voltage_violation"], m_r["voltage_violation"][i])
        with pytest.raises(RuntimeError):
            venv.reset_at(0)                     # lockstep: no mid-episode reset


def test_base_env_poll_send_episode_and_reset():
    """BaseEnv protocol over a whole episode: poll -> send_actions -> poll ...,
    done on the last step for every sub-env, then try_reset starts the next
    episode for the whole batch (equal to a batched reset)."""
    from powergridworld_amd.vector_env import MultiAgentVectorEnv
    n = 4
    ref, env = _pair(n, True)
    venv = MultiAgentVectorEnv(env)
    ref.reset()
    obs, rew, dones, infos, _ = venv.poll()
    assert set(obs) == set(range(n)) and all(d["__all__"] is False for d in dones.values())
    assert venv.poll()[0] == {}                  # nothing new until actions are sent
    rng = np.random.default_rng(6)
    steps = 0
    while True:
        act = _batched_actions(ref, rng, n)
        o_r, r_r, d_r, _ = ref.step(act)
        venv.send_actions({i: a for i, a in enumerate(_split(act, n))})
        obs, rew, dones, infos, _ = venv.poll()
        steps += 1
        for i in range(n):
            _eq(rew[i], {a: v[i] for a, v in r_r.items()})
            assert dones[i] == d_r
        if d_r["__all__"]:
            break
    assert steps == ref.max_episode_steps - 1 or steps == 286
    with pytest.raises(RuntimeError):
        venv.send_actions({i: a for i, a in enumerate(_split(_batched_actions(ref, rng, n), n))})
    o_ref = ref.reset()
    first = venv.try_reset(2)
    again = venv.try_reset(3)                    # the same boundary: no second reset
    _eq(first[2], {a: {c: v[2] for c, v in comps.items()} for a, comps in o_ref.items()})
    _eq(again[3], {a: {c: v[3] for c, v in comps.items()} for a, comps in o_ref.items()})


def test_poll_results_survive_the_next_step():
    """RLlib's collectors keep each step's observations until they build a
    batch: by default the adapter hands out rows of a per-step copy, so an
    earlier poll() result is not overwritten by the next step.  zero_copy=True
    hands out the engine's own buffers (valid until the next step)."""
    from powergridworld_amd.vector_env import MultiAgentVectorEnv
    n = 3
    for zero_copy in (False, True):
        ref, env = _pair(n, True)
        venv = MultiAgentVectorEnv(env, zero_copy=zero_copy)
        ref.reset()
        venv.poll()
        rng = np.random.default_rng(7)
        act1, act2 = _batched_actions(ref, rng, n), _batched_actions(ref, rng, n)
        venv.send_actions({i: a for i, a in enumerate(_split(act1, n))})
        obs1, rew1, _, _, _ = venv.poll()
        kept = {i: {a: {c: v.clone() for c, v in comps.items()} for a, comps in obs1[i].items()}
                for i in range(n)}
        kept_r = {i: {a: v.clone() for a, v in rew1[i].items()} for i in range(n)}
        venv.send_actions({i: a for i, a in enumerate(_split(act2, n))})
        obs2, _, _, _, _ = venv.poll()
        name = env.agents[0].name
        if zero_copy:      # the same engine buffer: now the second step's values
            assert obs1[0][name]["storage"].data_ptr() == obs2[0][name]["storage"].data_ptr()
        else:
            for i in range(n):
                _eq(obs1[i], kept[i])
                _eq(rew1[i], kept_r[i])
            assert not torch.equal(obs1[0][name]["building"], obs2[0][name]["building"])
