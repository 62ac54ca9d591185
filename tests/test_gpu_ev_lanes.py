"""Lanes over vehicles (pgw_ev_step_lanes): the EV step
with env-major requirements (N x pgw_ev_row(V)), LPE lanes per env and
butterfly sums, against the one-lane walk (pgw_ev_step, V x N) on the same
pre-step state, step info and actions over a whole episode -- the new
requirements, the charging bits and the vehicle counts equal bit for bit, the
sums (and so obs, real power, reward) within rounding of their order
(ev_charging_env.py:186-252 sums in vehicle order; the walk folds 8 groups of
chunks, the lanes a butterfly).  tools/gpu/ev_lanes_ab.py times the two
(profiles/r06/ev_lanes_ab.txt).  Needs an MI355X."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rows(x, row):
    V, n = x.shape
    out = torch.zeros((n, row), dtype=x.dtype, device=x.device)
    out[:, :V] = x.t()
    return out


@pytest.mark.parametrize("V,n,randomize", [(100, 4096, False), (25, 8192, False), (10, 4096, False),
                                           (40, 4096, True), (200, 2048, False)])
def test_ev_lanes_equal_the_walk(V, n, randomize):
    from powergridworld_amd import _lib
    from powergridworld_amd.agents import EVChargingEnv
    from powergridworld_amd.base import as_action
    lib = _lib.lib()
    env = EVChargingEnv(num_vehicles=V, minutes_per_step=5, max_charge_rate_kw=7., peak_threshold=250.,
                        vehicle_multiplier=5., rescale_spaces=True, randomize=randomize, num_envs=n, device=DEV)
    if randomize:
        env.seed(3)
    env.reset()
    row = int(lib.pgw_ev_row(V))
    assert row >= V and row in (16, 32) + tuple(64 * (1 << k) for k in range(5))
    st = _lib.stream_ptr(torch.device(DEV))
    gen = torch.Generator(DEV).manual_seed(V)
    est = _rows(env._env_start, row) if randomize else None
    een = _rows(env._env_endp, row) if randomize else None
    zeros = lambda: torch.zeros(n, dtype=torch.float64, device=DEV)
    steps = 0
    while not env.is_terminal():
        a = torch.rand((n, 1), dtype=torch.float64, device=DEV, generator=gen) * 2.4 - 1.2
        s = env._step_info_at(env.time_index, env._prev_window)[0]
        s1 = type(s).from_buffer_copy(s)
        if randomize:
            s1.env_start, s1.env_endp = est.data_ptr(), een.data_ptr()
        req0, chg0, obs0, rp0, rew0 = env.req.clone(), env.charging.clone(), env._new_obs(6), zeros(), zeros()
        req1, chg1, obs1, rp1, rew1 = _rows(env.req, row), env.charging.clone(), env._new_obs(6), zeros(), zeros()
        am = env._mat(as_action(a, n, 1, DEV, torch.float64))
        _lib.check(lib.pgw_ev_step(env.params, s, n, am, _lib.dptr(env._endp_dev), req0.data_ptr(), chg0.data_ptr(),
                                   env._mat(obs0), rp0.data_ptr(), rew0.data_ptr(), st))
        _lib.check(lib.pgw_ev_step_lanes(env.params, s1, n, am, _lib.dptr(env._endp_dev), req1.data_ptr(),
                                         chg1.data_ptr(), env._mat(obs1), rp1.data_ptr(), rew1.data_ptr(), st))
        torch.cuda.synchronize()
        assert torch.equal(req1[:, :V], req0.t()), steps
        assert torch.equal(chg1, chg0), steps
        assert torch.equal(obs1[:, 1], obs0[:, 1]), steps            # num_active_vehicles
        torch.testing.assert_close(obs1, obs0, rtol=1e-12, atol=1e-11)
        torch.testing.assert_close(rp1, rp0, rtol=1e-12, atol=1e-11)
        torch.testing.assert_close(rew1, rew0, rtol=1e-9, atol=1e-11)
        env.step(a)
        assert torch.equal(env.req, req0) and torch.equal(env._obs, obs0), steps
        steps += 1
    assert steps == 286                     # (the reset took the first of 287 step times)
