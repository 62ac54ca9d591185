"""Which layer of the OpenDSS-rule kernel's test decides each iteration on C4
loads (CPU, oracle; measurement infrastructure): per step and iteration, the
envs still iterating, those whose element nodes alone fail the test by the
square-root-free lower bound, those that need the exact test, and the waves
(64 envs) that run it.  Usage: python tools/od_test_layers.py"""
import sys, numpy as np
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.ma_oracle import CoordinatedOracle
from oracle.pf_oracle import BatchedPF
K = 2048
ora = CoordinatedOracle(K)
ora.pf = BatchedPF(system_load_rescale_factor=1.2, semantics="opendss")
f = ora.pf.feeder
cap = []
orig = f.snap_opendss
def hook(kw, kvar, *a, **k):
    cap.append((np.array(kw), np.array(kvar)))
    return orig(kw, kvar, *a, **k)
f.snap_opendss = hook
rng = np.random.default_rng(0)
ora.reset(rng.uniform(5.0, 45.0, size=(5, K)))
for t in range(12):
    ora.step(rng.uniform(-1, 1, size=(5, K, 8)))
C = f.Cinc; vbn = f.kv_ln * 1000.0
m = len(f.elem_p)
elem_nodes = sorted({int(f.elem_p[k]) for k in range(m) if f.elem_q[k] < 0})
ykw = np.asarray(f.base_kw, float)[f.elem_load] * 1000.0 / f.elem_nph
ykv = np.asarray(f.base_kvar, float)[f.elem_load] * 1000.0 / f.elem_nph
yeq = (ykw - 1j * ykv) / f.elem_vbase ** 2
Z = np.linalg.inv(f.Y + C.T @ np.diag(yeq) @ C)
print("step it active hit_all_elem(lower bound) need_exact waves_exact(of %d)" % (K // 64))
for s, (kw, kvar) in enumerate(cap[:12]):
    W_ph = kw[:, f.elem_load] * 1000.0 / f.elem_nph
    var_ph = kvar[:, f.elem_load] * 1000.0 / f.elem_nph
    V = (Z @ f.I_src)[None].repeat(kw.shape[0], 0)
    active = np.ones(kw.shape[0], bool)
    for it in range(1, 16):
        U = V @ C.T
        IL = f.load_currents(U, W_ph, var_ph)
        Vn = (f.I_src[None] + (yeq * U - IL) @ C) @ Z.T
        A2 = (np.abs(Vn[:, elem_nodes]) / vbn[elem_nodes]) ** 2
        B2 = (np.abs(V[:, elem_nodes]) / vbn[elem_nodes]) ** 2
        hit = (np.abs(A2 - B2) > 1e-4 * (0.5 * (A2 + B2) + 1)).any(1)
        err = np.max(np.abs(np.abs(Vn) - np.abs(V)) / vbn, axis=1)
        need = active & (it >= 2) & ~hit
        waves = need.reshape(-1, 64).any(1).sum()
        print(s, it, active.sum(), (active & hit).sum(), need.sum(), waves)
        conv = (err <= 1e-4) & (it >= 2)
        V = np.where(active[:, None], Vn, V)
        active &= ~conv
        if not active.any(): break
