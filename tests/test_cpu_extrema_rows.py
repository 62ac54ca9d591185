"""The extrema-row proof behind pgw_pf_od.resp_rows
(OpenDSSSolver._od_row_mask -> distribution_system.opendss.extrema_candidates):
on random pieces of complex quadratics V_r(t) = A + t (B + t C), the row
holding the minimum or the maximum |V| at any t of a dense grid inside each
piece is always among the candidates, and far-away rows are excluded."""
import numpy as np
import torch

from powergridworld_amd.distribution_system.opendss import extrema_candidates


def _pieces(rng, P, R, spread):
    base = 1.0 + spread * rng.standard_normal((1, R))               # rows at distinct levels
    A = base + 0.01 * rng.standard_normal((P, R)) + 1j * 0.05 * rng.standard_normal((P, R))
    B = 1e-3 * (rng.standard_normal((P, R)) + 1j * rng.standard_normal((P, R)))
    C = 1e-4 * (rng.standard_normal((P, R)) + 1j * rng.standard_normal((P, R)))
    tl = -rng.uniform(0.5, 1.0, P)
    th = rng.uniform(0.5, 1.0, P)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    return A, B, C, tl, th, T


def test_true_extrema_rows_are_candidates():
    rng = np.random.default_rng(0)
    for spread in (0.0, 0.003, 0.05):
        A, B, C, tl, th, T = _pieces(rng, 200, 38, spread)
        cand = extrema_candidates(T(A), T(B), T(C), T(tl), T(th))
        assert cand is not None
        t = tl[:, None] + (th - tl)[:, None] * np.linspace(0.0, 1.0, 513)[None, :]       # [P, 513]
        V = A[:, None, :] + t[:, :, None] * (B[:, None, :] + t[:, :, None] * C[:, None, :])
        m = np.abs(V)
        assert cand[np.unique(m.argmin(2))].all() and cand[np.unique(m.argmax(2))].all()
        if spread == 0.05:                    # well-separated rows: most are proved out
            assert cand.sum() < 20, cand.sum()


def test_nonfinite_bounds_keep_every_row():
    rng = np.random.default_rng(1)
    A, B, C, tl, th, T = _pieces(rng, 4, 6, 0.01)
    A[0, 2] = np.nan
    assert extrema_candidates(T(A), T(B), T(C), T(tl), T(th)) is None
