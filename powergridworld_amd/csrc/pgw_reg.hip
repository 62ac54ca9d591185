// RegControl on the general power flow (include/pgw.h, "RegControl"): the
// per-env Woodbury factor K(t) of the regulators' tap deviation and the
// control pass of OpenDSS's RegControl in STATIC mode.  Replaces what the
// OpenDSS engine does inside the reference's `Solve mode=snap`
// (gridworld/distribution_system/opendss.py:134) for a feeder file with
// RegControl objects (opendss.py:36-39 redirects any DSS file); the rules are
// restated from OpenDSS's published RegControl / SolveSnap documentation in
// oracle/pf_oracle.py (Feeder.solve_regulated), which the tests compare.
//
// Layout (gfx950): the factor is one wave per one or two envs -- lane j owns
// column j of the env's augmented [I + D S | D] (r <= 24 rows, 2r <= 48
// columns; two envs of 32 lanes each when 2r <= 32) in LDS,
// Gauss-Jordan with partial pivoting, the pivot column read into registers
// before the wave updates its columns; the control pass is one lane per env
// (a handful of complex multiply-adds per RegControl; Sample's options --
// PTphase=max / min, a remote regulated bus, Vlimit, inverse time -- are
// per-control branches on uniform settings).  Both are tiny next to
// the power flow itself: K is rebuilt only for the envs whose taps moved.
#include <cmath>

#include "pgw_common.h"

namespace pgw {

constexpr int kRegMax = PGW_PFG_MAX_REG;

struct c2 {
  double x, y;
};
__device__ __forceinline__ c2 cmul(c2 a, c2 b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ c2 cadd(c2 a, c2 b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ c2 csub(c2 a, c2 b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ c2 cscale(c2 a, double s) { return {a.x * s, a.y * s}; }

// The regulated phase's primitive admittance at taps (t1, t2) over (a, b).
__device__ __forceinline__ void reg_yprim(const pgw_reg_phase& ph, double t1, double t2, c2& yaa, c2& yab,
                                          c2& ybb) {
  yaa = cscale({ph.A[0], ph.A[1]}, 1.0 / (t1 * t1));
  yab = cscale({ph.B[0], ph.B[1]}, 1.0 / (t1 * t2));
  ybb = cscale({ph.C[0], ph.C[1]}, 1.0 / (t2 * t2));
}
__device__ __forceinline__ void reg_taps(const pgw_reg_phase& ph, double tap, double& t1, double& t2) {
  t1 = ph.tap_winding == 1 ? tap : ph.tap1;
  t2 = ph.tap_winding == 2 ? tap : ph.tap2;
}

// EPB envs per 64-lane block (2 when 2 r <= 32: lanes 32 h + j serve env 2b + h,
// column j), COLS = 64 / EPB columns per env; RMAX rows.
template <int EPB>
__global__ void __launch_bounds__(64) k_reg_factor(pgw_reg_params p_, int64_t n, const double* __restrict__ taps,
                                                   const int32_t* __restrict__ active, double* __restrict__ K) {
  constexpr int COLS = 64 / EPB;
  constexpr int RMAX = EPB == 2 ? 16 : kRegMax;
  const pgw_reg_params& p = PGW_KERNARG0(pgw_reg_params);
  const int lane = threadIdx.x, h = lane / COLS, jl = lane % COLS;
  const int64_t e = (int64_t)blockIdx.x * EPB + h;
  const bool live = e < n && (!active || active[e] != 0);
  if (!__syncthreads_or(live)) return;      // (uniform: every lane of the block takes it)
  const int64_t ec = e < n ? e : 0;
  const int r = p.r_reg;
  __shared__ c2 A[EPB * RMAX * COLS];        // env h: row i, column jl at A[(h RMAX + i) COLS + jl]
  c2* Ah = A + h * RMAX * COLS;
  // column jl of [I + D S | D] from the sparse D (a 2 x 2 block per regulated
  // phase over its nodes a, b): (D S)[i][j] = sum over the phases holding i of
  // D[i][a] S[a][j] + D[i][b] S[b][j]
  const c2* S = reinterpret_cast<const c2*>(p.S);
  const int j = jl < r ? jl : jl - r;
  const bool mcol = jl < r;
  c2 col[RMAX];
#pragma unroll
  for (int i = 0; i < RMAX; ++i) col[i] = {(mcol && i == j) ? 1.0 : 0.0, 0.0};
  for (int q = 0; q < p.n_phase; ++q) {
    const pgw_reg_phase& ph = p.phase[q];
    double t1, t2;
    reg_taps(ph, taps[(int64_t)ph.ctrl * n + ec], t1, t2);
    c2 aa, ab, bb, aa0, ab0, bb0;
    reg_yprim(ph, t1, t2, aa, ab, bb);
    reg_yprim(ph, ph.tap1, ph.tap2, aa0, ab0, bb0);
    const c2 daa = csub(aa, aa0), dab = csub(ab, ab0), dbb = csub(bb, bb0);
    const int a = ph.a, b = ph.b;
    c2 ta, tb;                                          // this column's entries of rows a, b
    if (mcol) {
      const c2 sa = S[a * r + j], sb = S[b * r + j];
      ta = cadd(cmul(daa, sa), cmul(dab, sb));
      tb = cadd(cmul(dab, sa), cmul(dbb, sb));
    } else {
      ta = (j == a) ? daa : (j == b ? dab : c2{0.0, 0.0});
      tb = (j == a) ? dab : (j == b ? dbb : c2{0.0, 0.0});
    }
#pragma unroll
    for (int i = 0; i < RMAX; ++i) {
      col[i] = (i == a) ? cadd(col[i], ta) : col[i];
      col[i] = (i == b) ? cadd(col[i], tb) : col[i];
    }
  }
#pragma unroll
  for (int i = 0; i < RMAX; ++i)
    if (i < r) Ah[i * COLS + jl] = (jl < 2 * r) ? col[i] : c2{0.0, 0.0};
  __syncthreads();
  bool singular = false;
  for (int c = 0; c < r; ++c) {
    // pivot: the largest |A[i][c]|, i >= c (every lane of the env finds the same row)
    int pr = c;
    double best = -1.0;
    for (int i = c; i < r; ++i) {
      const c2 v = Ah[i * COLS + c];
      const double a2 = v.x * v.x + v.y * v.y;
      if (a2 > best) {
        best = a2;
        pr = i;
      }
    }
    singular = singular || !(best > 0.0) || !isfinite(best);
    c2 pc[RMAX];                        // the pivot column, rows swapped
#pragma unroll
    for (int i = 0; i < RMAX; ++i) {
      const int src = (i == c) ? pr : (i == pr ? c : i);
      pc[i] = i < r ? Ah[src * COLS + c] : c2{0.0, 0.0};
    }
    const c2 rowc = Ah[pr * COLS + jl], rowp = Ah[c * COLS + jl];
    __syncthreads();                    // (all reads of column c done)
    // normalise the pivot row, eliminate the others (this lane's column)
    const c2 pv = pc[c];
    const double inv = 1.0 / (pv.x * pv.x + pv.y * pv.y);
    const c2 f = cmul(rowc, {pv.x * inv, -pv.y * inv});
#pragma unroll
    for (int i = 0; i < RMAX; ++i) {
      if (i < r) {
        c2 v;
        if (i == c) v = f;
        else {
          const c2 old = (i == pr) ? rowp : Ah[i * COLS + jl];
          v = csub(old, cmul(pc[i], f));
        }
        Ah[i * COLS + jl] = v;
      }
    }
    __syncthreads();
  }
  // K: columns r .. 2r - 1 hold (I + D S)^-1 D, complex symmetric (D and S
  // are); its upper triangle is stored (column jj: rows 0 .. jj), half the
  // bytes every solve iteration re-reads
  if (live && jl >= r && jl < 2 * r) {
    const int jj = jl - r;
    for (int i = 0; i <= jj; ++i) {
      const c2 v = Ah[i * COLS + jl];
      const int64_t o = 2 * ((int64_t)(i * r - i * (i - 1) / 2 + (jj - i)) * n + e);
      K[o] = singular ? NAN : v.x;
      K[o + 1] = singular ? NAN : v.y;
    }
  }
}

// V at regulator node j: x_j rho_j - sum_l S_jl c_l (c: the env's corrections, in registers).
__device__ __forceinline__ c2 reg_node_v(const pgw_reg_params& p, int j, const double* __restrict__ rx,
                                         const c2 (&c)[kRegMax], int64_t n, int64_t e) {
  const int r = p.r_reg;
  const c2* S = reinterpret_cast<const c2*>(p.S);
  c2 v = cscale({rx[2 * ((int64_t)j * n + e)], rx[2 * ((int64_t)j * n + e) + 1]}, p.rho[j]);
#pragma unroll
  for (int l = 0; l < kRegMax; ++l)
    if (l < r) v = csub(v, cmul(S[j * r + l], c[l]));
  return v;
}

__global__ void __launch_bounds__(kBlock) k_reg_control(pgw_reg_params p_, int64_t n, const double* __restrict__ rx,
                                                        const double* __restrict__ rc, double* __restrict__ taps,
                                                        int32_t* __restrict__ active, int32_t* __restrict__ n_changed) {
  const pgw_reg_params& p = PGW_KERNARG0(pgw_reg_params);
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  double want[PGW_REG_MAX_CTRL];
  double dmin = INFINITY;
  c2 c[kRegMax];
#pragma unroll
  for (int l = 0; l < kRegMax; ++l)
    c[l] = l < p.r_reg ? c2{rc[2 * ((int64_t)l * n + e)], rc[2 * ((int64_t)l * n + e) + 1]} : c2{0.0, 0.0};
  double dl[PGW_REG_MAX_CTRL];                       // each acting control's delay
  for (int g = 0; g < p.n_ctrl; ++g) {
    const pgw_reg_ctrl& C = p.ctrl[g];
    const double tap = taps[(int64_t)g * n + e];
    want[g] = tap;
    dl[g] = INFINITY;
    // RegControl.Sample: the monitored voltage -- the PT phase's, or with
    // PTphase=max / min the phase of largest / smallest |V| (the first on a
    // tie) -- on the 120-V base (V / PTratio)
    int k = 0;
    c2 vk = reg_node_v(p, C.mon_node[0], rx, c, n, e);
    double mk = sqrt(vk.x * vk.x + vk.y * vk.y);
    for (int i = 1; i < C.n_mon; ++i) {
      const c2 v = reg_node_v(p, C.mon_node[i], rx, c, n, e);
      const double mv = sqrt(v.x * v.x + v.y * v.y);
      if (C.pick == PGW_REG_PICK_MAX ? mv > mk : mv < mk) {
        k = i;
        vk = v;
        mk = mv;
      }
    }
    c2 vc = {vk.x / C.ptratio, vk.y / C.ptratio};
    // Vlimit: the local voltage -- the control voltage before LDC, or with a
    // regulated bus the winding's first phase (V / PTratio)
    double vlocal = 0.0;
    if (C.vlimit > 0.0) {
      if (C.vlim_node >= 0) {
        const c2 vl = reg_node_v(p, C.vlim_node, rx, c, n, e);
        vlocal = sqrt((vl.x / C.ptratio) * (vl.x / C.ptratio) + (vl.y / C.ptratio) * (vl.y / C.ptratio));
      } else {
        vlocal = sqrt(vc.x * vc.x + vc.y * vc.y);
      }
    }
    // the line-drop compensation (R + jX) I / CTprim, I the current the
    // controlled phase delivers from the monitored winding into its bus
    if (C.ldc) {
      const pgw_reg_phase& ph = p.phase[C.mon_phase[k]];
      double t1, t2;
      reg_taps(ph, tap, t1, t2);
      c2 yaa, yab, ybb;
      reg_yprim(ph, t1, t2, yaa, yab, ybb);
      const c2 va = reg_node_v(p, ph.a, rx, c, n, e), vb = reg_node_v(p, ph.b, rx, c, n, e);
      const c2 i_in = C.winding == 2 ? cadd(cmul(yab, va), cmul(ybb, vb)) : cadd(cmul(yaa, va), cmul(yab, vb));
      const c2 i_out = cscale(i_in, -1.0 / C.ctprim);
      vc = csub(vc, cmul({C.r_ldc, C.x_ldc}, i_out));
    }
    const double vact = sqrt(vc.x * vc.x + vc.y * vc.y);
    const double dv = C.vreg - vact;
    const bool over = C.vlimit > 0.0 && vlocal > C.vlimit;
    if (fabs(dv) > C.band * 0.5 || over) {
      // DoPendingAction (STATIC): the needed change (above Vlimit: down to it),
      // truncated to whole taps, at least one, at most max_tap_change, inside
      // [min_tap, max_tap]
      const double need = (over ? C.vlimit - vlocal : dv) / C.vbase;
      double steps = trunc(fabs(need) / C.incr);
      steps = fmin(fmax(steps, 1.0), (double)C.max_tap_change);
      double nt = tap + (need > 0.0 ? steps : -steps) * C.incr;
      nt = fmin(fmax(nt, C.min_tap), C.max_tap);
      if (nt != tap) {
        want[g] = nt;
        dl[g] = C.inverse_time ? C.delay / fmin(10.0, 2.0 * fabs(dv) / C.band) : C.delay;
        dmin = fmin(dmin, dl[g]);
      }
    }
  }
  // ControlQueue.DoNearestActions: only the actions with the smallest delay
  bool moved = false;
  for (int g = 0; g < p.n_ctrl; ++g) {
    const double tap = taps[(int64_t)g * n + e];
    if (want[g] != tap && dl[g] == dmin) {
      taps[(int64_t)g * n + e] = want[g];
      moved = true;
    }
  }
  active[e] = moved ? 1 : 0;
  if (moved && n_changed) atomicAdd(n_changed, 1);
}

}  // namespace pgw

using namespace pgw;

extern "C" {

static int32_t reg_check(const pgw_reg_params* p, const char* who) {
  PGW_REQUIRE(p && p->r_reg >= 1 && p->r_reg <= p->n_reg && p->n_reg <= PGW_PFG_MAX_REG && p->S && p->rho,
              "%s: bad regulator parameters", who);
  PGW_REQUIRE(p->n_phase >= 1 && p->n_phase <= PGW_REG_MAX_PHASES && p->n_ctrl >= 1 &&
                  p->n_ctrl <= PGW_REG_MAX_CTRL, "%s: %d phases / %d controls", who, p->n_phase, p->n_ctrl);
  for (int q = 0; q < p->n_phase; ++q) {
    const pgw_reg_phase& ph = p->phase[q];
    PGW_REQUIRE(ph.a >= 0 && ph.a < p->r_reg && ph.b >= 0 && ph.b < p->r_reg && ph.a != ph.b &&
                    ph.ctrl >= 0 && ph.ctrl < p->n_ctrl && (ph.tap_winding == 1 || ph.tap_winding == 2),
                "%s: regulated phase %d", who, q);
  }
  for (int g = 0; g < p->n_ctrl; ++g) {
    const pgw_reg_ctrl& C = p->ctrl[g];
    PGW_REQUIRE(C.n_mon >= 1 && C.n_mon <= PGW_REG_MAX_MON && C.pick >= PGW_REG_PICK_PHASE &&
                    C.pick <= PGW_REG_PICK_MIN && (C.pick != PGW_REG_PICK_PHASE || C.n_mon == 1) &&
                    (C.winding == 1 || C.winding == 2) && C.ptratio > 0.0 && C.ctprim > 0.0 && C.incr > 0.0 &&
                    C.vbase > 0.0 && C.min_tap <= C.max_tap && C.max_tap_change >= 1 && C.band > 0.0 &&
                    C.vlimit >= 0.0 && C.vlim_node >= -1 && C.vlim_node < p->r_reg,
                "%s: RegControl %d", who, g);
    for (int i = 0; i < C.n_mon; ++i)
      PGW_REQUIRE(C.mon_node[i] >= 0 && C.mon_node[i] < p->r_reg && C.mon_phase[i] >= 0 &&
                      C.mon_phase[i] < p->n_phase && p->phase[C.mon_phase[i]].ctrl == g,
                  "%s: RegControl %d monitored phase %d", who, g, i);
  }
  return PGW_OK;
}

int32_t pgw_reg_factor(const pgw_reg_params* p, int64_t n, const double* taps, const int32_t* active,
                       double* Kreg, void* stream) {
  const int32_t rc = reg_check(p, "pgw_reg_factor");
  if (rc) return rc;
  PGW_REQUIRE(taps && Kreg && n >= 0, "pgw_reg_factor: null argument");
  PGW_REQUIRE(2 * p->r_reg <= 64, "pgw_reg_factor: r_reg %d > 32", p->r_reg);
  if (n == 0) return PGW_OK;
  if (2 * p->r_reg <= 32)
    hipLaunchKernelGGL(k_reg_factor<2>, dim3((unsigned)((n + 1) / 2)), dim3(64), 0, (hipStream_t)stream, *p, n,
                       taps, active, Kreg);
  else
    hipLaunchKernelGGL(k_reg_factor<1>, dim3((unsigned)n), dim3(64), 0, (hipStream_t)stream, *p, n, taps, active,
                       Kreg);
  return check_launch("k_reg_factor");
}

int32_t pgw_reg_control(const pgw_reg_params* p, int64_t n, const double* reg_x, const double* reg_c,
                        double* taps, int32_t* active, int32_t* n_changed, void* stream) {
  const int32_t rc = reg_check(p, "pgw_reg_control");
  if (rc) return rc;
  PGW_REQUIRE(reg_x && reg_c && taps && active && n >= 0, "pgw_reg_control: null argument");
  if (n == 0) return PGW_OK;
  hipLaunchKernelGGL(k_reg_control, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, *p, n, reg_x, reg_c, taps, active, n_changed);
  return check_launch("k_reg_control");
}

}  // extern "C"
