"""Certificates for the OpenDSS-rule response table (pgw_pf_od.resp).

A response-table piece serves every env whose controllable kW P lies in its
interval with one iteration count k* and one quadratic J'(P).  That is right
only if OpenDSS's snap solve (opendss.py:131-135 -> ``Solve mode=snap``, as
the kernels restate it: od_solve in csrc/pgw_pf.hip) takes the same decisions
at EVERY P of the interval: the same load band for every element of every
iterate u_1 .. u_{k*-1} (the current law switches there) and the same outcome
of every stopping test (not converged at iterations 2 .. k*-1, converged at
k*).  The table builder finds pieces by probing signatures at a few points;
this module proves the decisions constant over the whole interval instead.

Method: first-order Taylor models in the piece's coordinate t in [-1, 1]
(P = c + r t).  Every complex quantity of the iteration is carried as
x(t) = a + b t + R with a rigorous bound |R| <= e; sums and matrix products
are exact on (a, b) and add |M| e; products, |x|^2, 1/|u|^2 and |x| add their
second-order terms to e (bounds below).  u_1 and iteration 1's currents are
affine in P (the start table), so they start with e = 0.  A decision is
certain when its margin's whole range clears the threshold by `delta`:

* band of element k of u_j: the range of |u_j,k|^2 must not reach any of
  vlow^2, vmin^2, vmax^2 within delta_band;
* stopping test at iteration i: converged for sure when every node's
  | |V_i| - |V_{i-1}| | is <= tol - delta_stop over the interval, not
  converged for sure when some node's is > tol + delta_stop.

delta (1e-12) is far above the kernels' rounding (~1e-15 relative per
iterate) and the certificate's own, so a certified interval gets the table's
decisions from the kernels' solve at every P in it.  Intervals that fail are
cut into equal parts (down to ``min_width`` kW): next to a breakpoint only a guard zone of
roughly delta / slope kW stays uncertified and goes to the solve; a narrow
excursion the probes stepped over (a band or stopping outcome that flips and
flips back between two probes) can never be certified, so the piece is cut
to its longest certified run and the rest goes to the solve.
"""
import numpy as np
import torch

FNV_BASIS = np.uint64(0xcbf29ce484222325)
FNV_PRIME = np.uint64(0x100000001b3)


class SnapModel:
    """The snap solve of od_solve with one controllable slot (Q = 0), per hour
    row: u_1 = u1b[h] + P u1P, iteration 1's currents J_0 = J0[h] + P jP (the
    start table pgw_pf_od.start, as stored), then per iteration
    J = (s g(|u|^2) - y0') u with s = s0[h] + P fr, u_next = u0 + W J, every
    node V = V0 + G J (pu).  All arrays complex128 / float64 torch tensors on
    one device; h indexes the first axis of u1b, J0 and s0."""

    def __init__(self, u1b, u1P, J0, jP, s0, fr, y0, u0, W, G, V0, lo2, mn2, mx2, tol, min_iter, max_iter):
        self.u1b, self.u1P, self.J0, self.jP = u1b, u1P, J0, jP
        self.s0, self.fr, self.y0, self.u0 = s0, fr, y0, u0
        self.W, self.G, self.V0 = W, G, V0
        self.Wa, self.Ga = W.abs(), G.abs()
        self.lo2, self.mn2, self.mx2 = float(lo2), float(mn2), float(mx2)
        self.tol, self.min_iter, self.max_iter = float(tol), int(min_iter), int(max_iter)

    @property
    def M(self):
        return self.u0.shape[0]

    @classmethod
    def from_solver(cls, s, rows, hours):
        """The model of OpenDSSSolver `s` (fast OpenDSS-rule kernels) for its
        start-table rows `rows` (hours `hours`)."""
        M, dev = s.M, s.device
        st = s._od_start[torch.as_tensor(rows, device=dev)].to(torch.float64)
        c = torch.view_as_complex(st.reshape(len(rows), 6, M, 2).contiguous())
        p0, od = s.params, s._od_proto
        nph = np.array(p0.nph[:M])
        ctrl0 = np.array(p0.elem_ctrl[:M]) == 0
        s0 = []
        for h in hours:
            p = s._params_for_hour(h)
            s0.append((np.array(p.base_kw[:M]) * 1000.0) / nph - 1j * ((np.array(p.base_kvar[:M]) * 1000.0) / nph))
        T = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)
        return cls(u1b=c[:, 0], u1P=c[0, 1], J0=c[:, 3], jP=c[0, 4], s0=T(np.array(s0)),
                   fr=T(np.where(ctrl0, 1000.0 / nph, 0.0)),
                   y0=T(np.array(od.y0r[:M]) + 1j * np.array(od.y0i[:M])), u0=T(s._od_u0),
                   W=T(s._od_W2), G=T(s._od_Gall[:, :M]), V0=T(s._od_V0all),
                   lo2=p0.vlow[0] ** 2, mn2=p0.vmin[0] ** 2, mx2=p0.vmax[0] ** 2,
                   tol=s.tol, min_iter=s.min_iter, max_iter=s.max_iter)

    # ---------------------------------------------------------------- points
    def bands_of(self, m2):
        return ((m2 > self.lo2).long() + (m2 > self.mn2).long() + (m2 > self.mx2).long())

    def solve_points(self, h, P):
        """The iteration at points (plain fp64, no bounds): (iterations [K]
        (negative: stopped by max_iter), signature [K] uint64 -- od_solve's
        SIG hash of every iterate's bands and the count).  For tests and the
        probes' restatement."""
        P = torch.as_tensor(P, dtype=torch.float64, device=self.u0.device)
        h = torch.as_tensor(h, device=self.u0.device)
        u = self.u1b[h] + P[:, None] * self.u1P
        Jp = self.J0[h] + P[:, None] * self.jP
        s = self.s0[h] + (P[:, None] * self.fr).to(torch.complex128)
        Vp = self.V0 + Jp @ self.G.T
        K = P.shape[0]
        done = torch.zeros(K, dtype=torch.bool, device=P.device)
        conv = torch.zeros_like(done)
        its = torch.ones(K, dtype=torch.int64, device=P.device)
        bands = []
        for it in range(2, self.max_iter + 1):
            m2 = u.real ** 2 + u.imag ** 2
            b = self.bands_of(m2)
            bands.append(torch.where(done, -1, (b << (2 * torch.arange(self.M, device=P.device))).sum(1)))
            mc = torch.where(m2 <= self.lo2, torch.ones_like(m2), m2.clamp(self.mn2, self.mx2))
            J = (s / mc - self.y0) * u
            V = self.V0 + J @ self.G.T
            u_n = self.u0 + J @ self.W.T
            err = (V.abs() - Vp.abs()).abs().max(1).values
            c_ = ~done & (it >= self.min_iter) & (err <= self.tol)
            its = torch.where(done, its, torch.full_like(its, it))
            conv |= c_
            done = done | c_ | (it >= self.max_iter)
            u, Vp = u_n, V                 # (a finished env's values are not read again)
            if bool(done.all()):
                break
        ret = torch.where(conv, its, -its)
        return ret, signature(torch.stack(bands, 1), ret)


def signature(bands, ret):
    """od_solve's SIG hash: per iteration the env runs, (sig ^ bands) * prime;
    then (sig ^ uint32(count)) * prime.  bands [K, iters] int64 (-1: not run)."""
    b = bands.cpu().numpy()
    r = ret.cpu().numpy().astype(np.int64)
    sig = np.full(b.shape[0], FNV_BASIS, np.uint64)
    with np.errstate(over="ignore"):
        for j in range(b.shape[1]):
            on = b[:, j] >= 0
            sig = np.where(on, (sig ^ b[:, j].astype(np.uint64)) * FNV_PRIME, sig)
        sig = (sig ^ (r & 0xffffffff).astype(np.uint64)) * FNV_PRIME
    return sig


# ------------------------------------------------------------- Taylor models
# x(t) = a + b t + R, t in [-1, 1], |R| <= e.  a, b complex [K, d]; e real [K, d].

def _lin(x, Mat, Mabs, const):
    a, b, e = x
    return const + a @ Mat.T, b @ Mat.T, e @ Mabs.T


def _mag2(x):
    """|x|^2 as a real model (m0 + m1 t + R, |R| <= em) and its range [lo, hi]."""
    a, b, e = x
    m0 = a.real ** 2 + a.imag ** 2
    m1 = 2.0 * (a.real * b.real + a.imag * b.imag)
    q2 = b.real ** 2 + b.imag ** 2
    qmax = m0 + m1.abs() + q2
    tv = torch.where(q2 > 0, -m1 / (2.0 * torch.where(q2 > 0, q2, torch.ones_like(q2))), torch.zeros_like(q2))
    inside = (q2 > 0) & (tv.abs() <= 1.0)
    qmin = torch.where(inside, m0 - m1 * m1 / (4.0 * torch.where(q2 > 0, q2, torch.ones_like(q2))),
                       m0 - m1.abs() + q2)
    qmin = qmin.clamp_min(0.0)
    rlo = (qmin.sqrt() - e).clamp_min(0.0)
    lo = rlo * rlo
    hi = (qmax.sqrt() + e) ** 2
    em = q2 + 2.0 * (a.abs() + b.abs()) * e + e * e
    return m0, m1, em, lo, hi


def _mag(x):
    """|x| as a real model: (mag0, slope, rem); rem = inf where |a| <= |b|."""
    a, b, e = x
    aa, ba = a.abs(), b.abs()
    slope = (a.real * b.real + a.imag * b.imag) / torch.where(aa > 0, aa, torch.ones_like(aa))
    gap = aa - ba
    rem = torch.where(gap > 0, e + ba * ba / (2.0 * torch.where(gap > 0, gap, torch.ones_like(gap))),
                      torch.full_like(aa, float("inf")))
    return aa, slope, rem


def _mul_cr(sa, sb, g0, g1, eg):
    """complex affine (sa + sb t) times real model (g0 + g1 t + G)."""
    a = sa * g0
    b = sa * g1 + sb * g0
    e = sb.abs() * g1.abs() + (sa.abs() + sb.abs()) * eg
    return a, b, e


def _mul_cc(x, y):
    xa, xb, xe = x
    ya, yb, ye = y
    a = xa * ya
    b = xa * yb + xb * ya
    e = xb.abs() * yb.abs() + (xa.abs() + xb.abs()) * ye + (ya.abs() + yb.abs()) * xe + xe * ye
    return a, b, e


def certify(model, h, lo, hi, delta_band=1e-12, delta_stop=1e-12):
    """Certify intervals [lo, hi] (kW) of hour rows h: returns (ok [K] bool,
    iterations [K] int64, signature [K] uint64).  ok means every band and
    stopping decision of the snap solve is the same at every P in the interval
    (then iterations / signature are its decisions)."""
    dev = model.u0.device
    h = torch.as_tensor(h, device=dev)
    lo = torch.as_tensor(lo, dtype=torch.float64, device=dev)
    hi = torch.as_tensor(hi, dtype=torch.float64, device=dev)
    K, M = lo.shape[0], model.M
    c, r = (0.5 * (lo + hi))[:, None], (0.5 * (hi - lo))[:, None]
    zero_e = torch.zeros((K, M), dtype=torch.float64, device=dev)
    u = (model.u1b[h] + c * model.u1P, r * model.u1P, zero_e)
    Jp = (model.J0[h] + c * model.jP, r * model.jP, zero_e)
    Vp = _lin(Jp, model.G, model.Ga, model.V0)
    s_a = model.s0[h] + (c * model.fr).to(torch.complex128)
    s_b = (r * model.fr).to(torch.complex128)
    ok = torch.ones(K, dtype=torch.bool, device=dev)
    done = torch.zeros(K, dtype=torch.bool, device=dev)
    conv = torch.zeros_like(done)
    its = torch.ones(K, dtype=torch.int64, device=dev)
    shifts = 2 * torch.arange(M, device=dev)
    thr = (model.lo2, model.mn2, model.mx2)
    bands = []
    for it in range(2, model.max_iter + 1):
        # ---- the bands of u_{it-1}: certain, or the interval fails
        m0, m1, em, mlo, mhi = _mag2(u)
        b = torch.zeros((K, M), dtype=torch.int64, device=dev)
        for T in thr:
            above, below = mlo > T + delta_band, mhi < T - delta_band
            ok &= done | (above | below).all(1)
            b += above.long()
        bands.append(torch.where(done, -1, (b << shifts).sum(1)))
        # ---- g = 1 / clamp(|u|^2) per band, as a real model
        inband = b == 2
        safe = torch.where(inband, m0, torch.ones_like(m0))
        g0 = torch.where(inband, 1.0 / safe,
                         torch.where(b == 1, 1.0 / model.mn2, torch.where(b == 3, 1.0 / model.mx2, 1.0)))
        g1 = torch.where(inband, -m1 / (safe * safe), torch.zeros_like(m1))
        mlo_s = torch.where(inband, mlo, torch.ones_like(mlo))
        eg = torch.where(inband, em / (safe * safe) + (m1.abs() + em) ** 2 / (safe * safe * mlo_s),
                         torch.zeros_like(em))
        ok &= done | torch.isfinite(eg).all(1)
        ya, yb, ye = _mul_cr(s_a, s_b, g0, g1, eg)
        J = _mul_cc((ya - model.y0, yb, ye), u)
        V = _lin(J, model.G, model.Ga, model.V0)
        un = _lin(J, model.W, model.Wa, model.u0)
        # ---- the stopping test: every node's | |V_it| - |V_it-1| | against tol
        n0, n1, nr = _mag(V)
        p0, p1, pr = _mag(Vp)
        d0, d1, dr = n0 - p0, n1 - p1, nr + pr
        dlo, dhi = d0 - d1.abs() - dr, d0 + d1.abs() + dr
        amax = torch.maximum(dlo.abs(), dhi.abs())
        amin = torch.where((dlo <= 0) & (dhi >= 0), torch.zeros_like(dlo), torch.minimum(dlo.abs(), dhi.abs()))
        if it >= model.min_iter:
            yes = (amax <= model.tol - delta_stop).all(1)
            no = (amin > model.tol + delta_stop).any(1)
        else:
            yes = torch.zeros_like(done)
            no = torch.ones_like(done)
        ok &= done | yes | no
        its = torch.where(done, its, torch.full_like(its, it))
        conv |= ~done & yes
        done = done | yes | (it >= model.max_iter) | ~ok
        u = tuple(torch.where(done[:, None], x_o, x_n) for x_o, x_n in zip(u, un))
        Vp = V
        if bool(done.all()):
            break
    ret = torch.where(conv, its, -its)
    return ok.cpu().numpy(), ret.cpu().numpy(), signature(torch.stack(bands, 1), ret)


def certify_pieces(model, h, a, b, it, sig, min_width=1e-9, max_depth=12, max_live=64, split=16):
    """The certified part of each piece [a, b] of hour row h whose table
    decisions are (it, sig): intervals that fail are cut into `split` equal
    parts (while wider than min_width, at most max_live failing intervals of one
    piece per level; split 16 reaches 1e-9 kW from 0.625 kW in 8 levels) and
    the piece keeps its longest run of certified intervals.  Returns (lo, hi,
    certified_kw) per piece; lo > hi when nothing is certified."""
    h, a, b = np.asarray(h), np.asarray(a, float), np.asarray(b, float)
    it, sig = np.asarray(it, np.int64), np.asarray(sig, np.uint64)
    n = len(a)
    out_lo, out_hi, kw = np.full(n, np.inf), np.full(n, -np.inf), np.zeros(n)
    if n == 0:
        return out_lo, out_hi, kw
    owner, lo, hi = np.arange(n), a.copy(), b.copy()
    good = {}
    for level in range(max_depth):
        if not len(owner):
            break
        ok, ret, sg = certify(model, h[owner], lo, hi)
        ok &= (ret == it[owner]) & (sg == sig[owner])
        if level == 0:                      # whole pieces certified at once: the usual case
            out_lo[ok], out_hi[ok], kw[ok] = a[ok], b[ok], b[ok] - a[ok]
        else:
            for q in np.nonzero(ok)[0]:
                good.setdefault(owner[q], []).append((lo[q], hi[q]))
        bad = np.nonzero(~ok & (hi - lo > split * min_width))[0]
        if max_live:
            keep, count = [], {}
            for q in bad:
                count[owner[q]] = count.get(owner[q], 0) + 1
                if count[owner[q]] <= max_live:
                    keep.append(q)
            bad = np.array(keep, np.int64)
        # the parts' edges computed once, so neighbours share them exactly
        edges = lo[bad, None] + (hi - lo)[bad, None] * (np.arange(split + 1) / split)[None, :]
        edges[:, -1] = hi[bad]
        owner = np.repeat(owner[bad], split)
        lo, hi = edges[:, :-1].ravel(), edges[:, 1:].ravel()
    for p, iv in good.items():
        iv = sorted(iv)
        kw[p] = sum(y - x for x, y in iv)
        best, cur = None, [iv[0][0], iv[0][1]]
        for x, y in iv[1:]:
            if x == cur[1]:
                cur[1] = y
            else:
                if best is None or cur[1] - cur[0] > best[1] - best[0]:
                    best = tuple(cur)
                cur = [x, y]
        if best is None or cur[1] - cur[0] > best[1] - best[0]:
            best = tuple(cur)
        out_lo[p], out_hi[p] = best
    return out_lo, out_hi, kw
