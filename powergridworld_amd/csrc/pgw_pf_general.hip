// General batched distribution power flow (pgw_pf_solve_general): any feeder
// size up to PGW_PFG_MAX_M load phase elements, and two stopping rules --
// the fixed point (PGW_PF_EXACT, as pgw_pf_solve) or OpenDSS's own snap solve
// (PGW_PF_OPENDSS).  Replaces OpenDSSSolver.calculate_power_flow
// (gridworld/distribution_system/opendss.py:80-165); the OpenDSS semantics
// follow its published solution method (Solution.pas SolveSnap ->
// DoNormalSolution, Load.CalcInjCurrentArray), restated in
// oracle/pf_oracle.py:Feeder.snap_opendss.
//
// Per env the solve iterates on the m load-element voltages in per unit of
// each element's base, u_i = u0_i + sum_k W''_ik I'_k(u_k), with
//   I'_k = (conj(S_k) g(|u_k|) - y0'_k) u_k,
//   g = 1/clamp(|u|^2, vmin^2, vmax^2), or 1 at or below vlow (Load model 1),
// y0' = 0 for the exact fixed point and the per-phase power of the Yeq that
// sits in OpenDSS's Y for its iteration (the compensation current).
//
// Layout (gfx950): a block of 4 waves serves 64 envs, lane = env.  The rows --
// m element rows, the OpenDSS check rows (every node) and the output rows --
// are cut into chunks of 8 and dealt round-robin to the waves; a wave keeps its
// element rows' voltages and its check rows' previous magnitudes in registers
// across iterations.  Per iteration every wave writes the currents of its
// element rows to LDS (J[k][lane], 16 B per element and env), the block
// synchronises, and every row accumulates sum_k M[k][row] J_k with the matrix
// entries as wave-uniform scalar operands (scalar loads through the constant
// cache: one s_load per 8 entries, reused by the 64 envs of the wave) and J_k
// from LDS (one ds_read_b128 per element, reused by the 8 rows of the chunk).
// Per-env convergence is the max over the waves' partial errors (LDS), and
// the loop runs until every env of the block has stopped; an env that stopped
// keeps its voltages, magnitudes and currents (selects), so its result and
// iteration count are those of solving it alone.
#include <cmath>

#include "pgw_common.h"

namespace pgw {

constexpr int kGW = kBlock / 64;   // waves per block (4)
constexpr int kGR = 8;             // rows per chunk

typedef const __attribute__((address_space(4))) double* cdptr;
typedef const __attribute__((address_space(4))) pgw_pfg_elem* ceptr;

// An element record through the scalar cache (field by field: no aggregate
// copies out of the constant address space).
struct ElemV {
  double base_kw, base_kvar, nph, y0r, y0i, vlo2, vmn2, vmx2;
  int ctrl, model;
};
__device__ __forceinline__ ElemV ld_elem(ceptr el, int k) {
  ElemV v;
  v.base_kw = el[k].base_kw;
  v.base_kvar = el[k].base_kvar;
  v.nph = el[k].nph;
  v.y0r = el[k].y0r;
  v.y0i = el[k].y0i;
  v.vlo2 = el[k].vlo2;
  v.vmn2 = el[k].vmn2;
  v.vmx2 = el[k].vmx2;
  v.ctrl = el[k].ctrl;
  v.model = el[k].model;
  return v;
}

__device__ __forceinline__ double g_rcp(double m) {
  double r = __builtin_amdgcn_rcp(m);   // v_rcp_f64 + two Newton steps (~1 ulp)
  double e = fma(-m, r, 1.0);
  r = fma(r, e, r);
  e = fma(-m, r, 1.0);
  return fma(r, e, r);
}

// The current-law coefficients (f_P, f_Q) of a load element of model != 1 at
// |u|^2 = m2: S(v) = P0 v^2 f_P + j Q0 v^2 f_Q, i.e. the factors of the nominal
// admittance per part (oracle/pf_oracle.py Feeder.LAWS):
//   band  1 / clamp(v^2, vmin^2, vmax^2)   z  1   i  1 / v   fixed  1 / v^2
//   exp   v^(k - 2)                        zip  Z + I / v + P / v^2
// every law but ZIP at the nominal admittance (1) at or below vlow; ZIP loads
// off (0) below their cutoff.  Model 1 stays on its own inline path.
__device__ __forceinline__ void elem_law(ceptr el, int k, const ElemV& E, double m2, double& fp,
                                         double& fq) {
  const int md = E.model;
  const double v = sqrt(m2);
  const double band = g_rcp(fmin(fmax(m2, E.vmn2), E.vmx2));
  if (md == 8) {
    const double zp = el[k].zip[0], ip = el[k].zip[1], pp = el[k].zip[2];
    const double zq = el[k].zip[3], iq = el[k].zip[4], pq = el[k].zip[5];
    const bool off = m2 < el[k].vcut2;
    fp = off ? 0.0 : (zp + ip / v) + pp / m2;
    fq = off ? 0.0 : (zq + iq / v) + pq / m2;
    return;
  }
  if (md == 4) {
    fp = pow(v, el[k].exp_p - 2.0);
    fq = pow(v, el[k].exp_q - 2.0);
  } else if (md == 5) {
    fp = fq = 1.0 / v;
  } else {                         // 3, 7: band P, constant-Z Q; 6: band P, fixed Q
    fp = band;
    fq = md == 6 ? 1.0 / m2 : 1.0;
  }
  const bool low = m2 <= E.vlo2;
  fp = low ? 1.0 : fp;
  fq = low ? 1.0 : fq;
}

// NaN-propagating max (an env whose error is NaN never converges).
__device__ __forceinline__ double nmax(double a, double b) { return (b > a || b != b) ? b : a; }

// One chunk of 8 rows: acc_r = base_r + sum_k M[k][row0 + r] J_k (complex).
// Matrices and bases are padded to whole chunks (zero rows), so no guards.
__device__ __forceinline__ void chunk_rows(cdptr M, int ld, int row0, cdptr base, int m,
                                           const double2* __restrict__ sJ, int lane,
                                           double (&ar)[kGR], double (&ai)[kGR]) {
#pragma unroll
  for (int r = 0; r < kGR; ++r) {
    ar[r] = base[2 * (row0 + r)];
    ai[r] = base[2 * (row0 + r) + 1];
  }
  for (int k = 0; k < m; ++k) {
    const double2 j = sJ[k * 64 + lane];
    const cdptr w = M + 2 * ((int64_t)k * ld + row0);
#pragma unroll
    for (int r = 0; r < kGR; ++r) {
      const double wr = w[2 * r], wi = w[2 * r + 1];
      ar[r] = fma(wr, j.x, ar[r]);
      ar[r] = fma(-wi, j.y, ar[r]);
      ai[r] = fma(wr, j.y, ai[r]);
      ai[r] = fma(wi, j.x, ai[r]);
    }
  }
}

// CE: element chunks per wave (m + n_reg <= 32 CE); CN: check chunks per wave
// (OpenDSS mode, n_chk <= 32 CN; 0 = exact mode); REG: regulators with
// per-env taps (pgw_pfg_params.n_reg > 0).
//
// REG: the sJ columns m .. m + n_reg - 1 hold the env's correction currents c
// (pgw.h).  Each pass: the currents J of the element rows -> LDS; the x rows
// (the DSS-tap voltages at the regulator nodes, x = V0reg + Greg J) -> LDS;
// c = K x per env (K from HBM, rows dealt to the waves) -> sJ; then every row
// as before over m + n_reg columns.  A first pass with J = 0 starts the solve
// from the direct solution at the env's taps (the element voltages and, for
// OpenDSS, the check rows' magnitudes), unless U_init is given.
template <int CE, int CN, bool REG>
__global__ void __launch_bounds__(kBlock) k_pf_general(pgw_pfg_params p, pgw_pfg_tables t, int64_t n,
                                                       const double* __restrict__ ctrl_p,
                                                       const double* __restrict__ ctrl_q,
                                                       double* __restrict__ v_out,
                                                       int32_t* __restrict__ iters, PFGCoord c) {
  constexpr bool OD = CN > 0;
  constexpr int kMaxRows = 32 * CE;
  __shared__ double2 sJ[kMaxRows * 64];
  __shared__ double2 s_x[REG ? PGW_PFG_MAX_REG * 64 : 1];
  __shared__ double s_err[kGW * 64];
  __shared__ double s_mn[kGW * 64], s_mx[kGW * 64], s_vsel[64];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t e = (int64_t)blockIdx.x * 64 + lane;
  const bool valid = e < n && (!t.env_active || t.env_active[e < n ? e : 0] != 0);
  const int64_t ec = e < n ? e : 0;
  const int m = p.m;
  const int mtot = REG ? m + p.n_reg : m;     // columns of W / Gc / G
  const ceptr el = (ceptr)t.elem;
  const cdptr W = (cdptr)t.W, U0 = (cdptr)t.U0;
  const bool step_yeq = p.mode == PGW_PF_OPENDSS_STEP;     // (uniform)

  // ---- the env's controllable powers (kW, kvar) per slot
  double cp[PGW_PF_MAX_CTRL], cq[PGW_PF_MAX_CTRL];
#pragma unroll
  for (int s = 0; s < PGW_PF_MAX_CTRL; ++s) {
    cp[s] = 0.0;
    cq[s] = 0.0;
  }
  if (c.agent_power) {
    // 0 + a0 + a1 ... per bus, in agent order (the generic path's sums)
#pragma unroll
    for (int ag = 0; ag < PGW_MAX_AGENTS; ++ag) {
      if (ag < c.n_agents) {
        const double x = valid ? c.agent_power[(int64_t)ag * n + ec] : 0.0;
        const int slot = c.agent_ctrl[ag];
#pragma unroll
        for (int s = 0; s < PGW_PF_MAX_CTRL; ++s) cp[s] = (s == slot) ? cp[s] + x : cp[s];
      }
    }
  } else {
#pragma unroll
    for (int s = 0; s < PGW_PF_MAX_CTRL; ++s) {
      if (s < p.n_ctrl) {
        cp[s] = (valid && ctrl_p) ? ctrl_p[(int64_t)s * n + ec] : 0.0;
        cq[s] = (valid && ctrl_q) ? ctrl_q[(int64_t)s * n + ec] : 0.0;
      }
    }
  }

  // ---- owned element rows: powers conj(S) (W, var) and the initial voltages
  double sr[CE][kGR], si[CE][kGR], ur[CE][kGR], ui[CE][kGR];
#pragma unroll
  for (int j = 0; j < CE; ++j) {
    const int row0 = (wv + kGW * j) * kGR;
#pragma unroll
    for (int r = 0; r < kGR; ++r) {
      const int k = row0 + r;
      sr[j][r] = si[j][r] = ur[j][r] = ui[j][r] = 0.0;
      if (k < m) {
        const ElemV E = ld_elem(el, k);
        double pk = 0.0, qk = 0.0;
#pragma unroll
        for (int s = 0; s < PGW_PF_MAX_CTRL; ++s) {
          pk = (E.ctrl == s) ? cp[s] : pk;
          qk = (E.ctrl == s) ? cq[s] : qk;
        }
        // opendss.py:107-108 (coef * base * rescale), :128-129 (+ controllable),
        // then OpenDSS WNominal = kW * 1000 / nphases; loads of other models
        // keep the DSS file's kW / kvar (the reference re-sets model 1 only)
        const bool pq = E.model == 1;
        const double kw = pq ? (p.coef * E.base_kw) * p.rescale : E.base_kw;
        const double kvar = pq ? (p.coef * E.base_kvar) * p.rescale : E.base_kvar;
        sr[j][r] = ((kw + pk) * 1000.0) / E.nph;
        si[j][r] = -(((kvar + qk) * 1000.0) / E.nph);
        if (t.U_init) {
          ur[j][r] = t.U_init[2 * (ec * m + k)];
          ui[j][r] = t.U_init[2 * (ec * m + k) + 1];
        } else {
          ur[j][r] = U0[2 * k];
          ui[j][r] = U0[2 * k + 1];
        }
      }
    }
  }
  // OpenDSS: the check rows' magnitudes of the previous iterate (the direct
  // solution before the first iteration; the test only counts from min_iter)
  double old[CN > 0 ? CN : 1][kGR];
  if constexpr (OD) {
    const cdptr V0c = (cdptr)t.V0c;
#pragma unroll
    for (int j = 0; j < CN; ++j) {
      const int row0 = (wv + kGW * j) * kGR;
#pragma unroll
      for (int r = 0; r < kGR; ++r) {
        const int o = row0 + r;
        old[j][r] = 0.0;
        if (o < p.n_chk) {
          const double vr = V0c[2 * o], vi = V0c[2 * o + 1];
          old[j][r] = sqrt(fma(vi, vi, vr * vr));
        }
      }
    }
  }

  const double tol2 = p.tol * p.tol;
  int it = 0, my_it = 0;
  bool done = !valid, conv_ok = !valid;
  bool first = REG && !t.U_init;     // REG: the direct-solution pass (J = 0) first
  while (true) {
    // ---- 1. currents of the owned element rows -> LDS (a stopped env keeps its last)
#pragma unroll
    for (int j = 0; j < CE; ++j) {
      const int row0 = (wv + kGW * j) * kGR;
      if (row0 < m) {
#pragma unroll
        for (int r = 0; r < kGR; ++r) {
          const int k = row0 + r;
          const ElemV E = ld_elem(el, min(k, m - 1));
          const double m2 = fma(ui[j][r], ui[j][r], ur[j][r] * ur[j][r]);
          double fp, fq;
          if (E.model == 1) {          // constant PQ (Load.DoConstantPQLoad)
            double mc = fmin(fmax(m2, E.vmn2), E.vmx2);
            mc = (m2 <= E.vlo2) ? 1.0 : mc;
            fp = fq = g_rcp(mc);
          } else {
            elem_law(el, min(k, m - 1), E, m2, fp, fq);
          }
          // (PGW_PF_OPENDSS_STEP: the Yeq in Y is the step's own power)
          const double y0r = step_yeq ? sr[j][r] : E.y0r, y0i = step_yeq ? si[j][r] : E.y0i;
          const double cr = OD ? fma(sr[j][r], fp, -y0r) : sr[j][r] * fp;
          const double ci = OD ? fma(si[j][r], fq, -y0i) : si[j][r] * fq;
          double jr = fma(cr, ur[j][r], -(ci * ui[j][r]));
          double ji = fma(cr, ui[j][r], ci * ur[j][r]);
          if (REG && first) jr = ji = 0.0;
          if (!done && k < m) sJ[k * 64 + lane] = make_double2(jr, ji);
        }
      }
    }
    __syncthreads();
    if constexpr (REG) {
      // ---- 1b. x rows (DSS-tap voltages at the regulator nodes) -> LDS
      for (int row0 = wv * kGR; row0 < p.n_reg; row0 += kGW * kGR) {
        double ar[kGR], ai[kGR];
        chunk_rows((cdptr)t.Greg, p.n_reg, row0, (cdptr)t.V0reg, m, sJ, lane, ar, ai);
#pragma unroll
        for (int r = 0; r < kGR; ++r) s_x[(row0 + r) * 64 + lane] = make_double2(ar[r], ai[r]);
      }
      __syncthreads();
      // ---- 1c. c = K (rho x) per env -> the correction columns of sJ (K
      // symmetric, its upper triangle stored: row jr0 reads column jr0 below
      // the diagonal).  A row's entries are loaded 8 at a time before their
      // FMAs (one HBM round trip per 8 columns, not per column); the FMAs run
      // in column order.
      const int rr = p.r_reg;
      for (int jr0 = wv; jr0 < rr; jr0 += kGW) {
        double cr_ = 0.0, ci_ = 0.0;
        for (int l0 = 0; l0 < rr; l0 += 8) {
          double kx[8], ky[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int l = min(l0 + u, rr - 1);          // (past the row: a valid address, value unused)
            const int i0 = min(jr0, l), i1 = max(jr0, l);
            const double* kp = t.Kreg + 2 * ((int64_t)(i0 * rr - i0 * (i0 - 1) / 2 + (i1 - i0)) * n + ec);
            kx[u] = kp[0];
            ky[u] = kp[1];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int l = l0 + u;
            if (l < rr) {
              const double2 xu = s_x[l * 64 + lane];
              const double rl = t.reg_rho[l];
              const double xr = xu.x * rl, xi = xu.y * rl;
              cr_ = fma(kx[u], xr, cr_);
              cr_ = fma(-ky[u], xi, cr_);
              ci_ = fma(kx[u], xi, ci_);
              ci_ = fma(ky[u], xr, ci_);
            }
          }
        }
        if (!done) sJ[(m + jr0) * 64 + lane] = make_double2(cr_, ci_);
      }
      for (int jr0 = rr + wv; jr0 < p.n_reg; jr0 += kGW) sJ[(m + jr0) * 64 + lane] = make_double2(0.0, 0.0);
      __syncthreads();
    }
    // ---- 2. new element voltages; OpenDSS: every node's magnitude change
    double err = 0.0;
#pragma unroll
    for (int j = 0; j < CE; ++j) {
      const int row0 = (wv + kGW * j) * kGR;
      if (row0 < m) {
        double ar[kGR], ai[kGR];
        chunk_rows(W, m, row0, U0, mtot, sJ, lane, ar, ai);
#pragma unroll
        for (int r = 0; r < kGR; ++r) {
          if (!OD) {
            const double dr = ar[r] - ur[j][r], di = ai[r] - ui[j][r];
            err = nmax(err, fma(dr, dr, di * di));
          }
          ur[j][r] = done ? ur[j][r] : ar[r];
          ui[j][r] = done ? ui[j][r] : ai[r];
        }
      }
    }
    if constexpr (OD) {
#pragma unroll
      for (int j = 0; j < CN; ++j) {
        const int row0 = (wv + kGW * j) * kGR;
        if (row0 < p.n_chk) {
          double ar[kGR], ai[kGR];
          chunk_rows((cdptr)t.Gc, p.n_chk, row0, (cdptr)t.V0c, mtot, sJ, lane, ar, ai);
#pragma unroll
          for (int r = 0; r < kGR; ++r) {
            const double mag = sqrt(fma(ai[r], ai[r], ar[r] * ar[r]));
            err = nmax(err, fabs(mag - old[j][r]));
            old[j][r] = done ? old[j][r] : mag;
          }
        }
      }
    }
    if (REG && first) {                // the start is set; the iterations begin
      first = false;
      __syncthreads();
      continue;
    }
    s_err[wv * 64 + lane] = err;
    __syncthreads();
    // ---- 3. per-env test (every wave forms the same value for its lane)
    double E = s_err[lane];
#pragma unroll
    for (int w = 1; w < kGW; ++w) E = nmax(E, s_err[w * 64 + lane]);
    ++it;
    const bool conv = OD ? (E <= p.tol && it >= p.min_iter) : (E < tol2);
    my_it = done ? my_it : it;
    conv_ok = conv_ok || (!done && conv);
    done = done || conv || it >= p.max_iter;
    // (also the barrier between this iteration's s_err / J reads and the next writes)
    if (!__syncthreads_or(!done)) break;
  }

  // ---- outputs: element voltages, then the output rows from each env's last
  // currents (the node voltages of the accepted solve, V = V0 + G I(u_prev))
  if (valid && t.U_out) {
#pragma unroll
    for (int j = 0; j < CE; ++j) {
      const int row0 = (wv + kGW * j) * kGR;
#pragma unroll
      for (int r = 0; r < kGR; ++r) {
        const int k = row0 + r;
        if (k < m) {
          t.U_out[2 * (e * m + k)] = ur[j][r];
          t.U_out[2 * (e * m + k) + 1] = ui[j][r];
        }
      }
    }
  }
  const int n_out = p.n_out;
  const int ld_out = (n_out + kGR - 1) / kGR * kGR;
  double vmn = INFINITY, vmx = -INFINITY, vsel = 0.0;
  bool have = false;
  for (int row0 = wv * kGR; row0 < n_out; row0 += kGW * kGR) {
    double ar[kGR], ai[kGR];
    chunk_rows((cdptr)t.G, ld_out, row0, (cdptr)t.V0, mtot, sJ, lane, ar, ai);
#pragma unroll
    for (int r = 0; r < kGR; ++r) {
      const int o = row0 + r;
      if (o < n_out) {
        const double v = sqrt(fma(ai[r], ai[r], ar[r] * ar[r]));
        if (valid && v_out) v_out[(int64_t)o * n + e] = v;
        // Python min()/max() over the rows in order: first strict improvement
        if (!have) {
          vmn = vmx = v;
          have = true;
        } else {
          vmn = (v < vmn) ? v : vmn;
          vmx = (v > vmx) ? v : vmx;
        }
        if (o == c.vv_row) vsel = v;
      }
    }
  }
  if (REG && valid) {                // the control pass's inputs: x and c of the accepted solve
    for (int j = wv; j < p.r_reg; j += kGW) {
      const double2 x = s_x[j * 64 + lane], cc = sJ[(m + j) * 64 + lane];
      t.reg_x[2 * ((int64_t)j * n + e)] = x.x;
      t.reg_x[2 * ((int64_t)j * n + e) + 1] = x.y;
      t.reg_c[2 * ((int64_t)j * n + e)] = cc.x;
      t.reg_c[2 * ((int64_t)j * n + e) + 1] = cc.y;
    }
  }
  // chunk q is wave q % 4's: rows in order across waves = chunks in order, so
  // the waves' extrema combine in wave order of their first chunks
  s_mn[wv * 64 + lane] = have ? vmn : NAN;
  s_mx[wv * 64 + lane] = have ? vmx : NAN;
  if (c.agent_power && ((c.vv_row / kGR) % kGW) == wv) s_vsel[lane] = vsel;
  __syncthreads();
  if (wv != 0 || !valid) return;
  if (t.v_min_out || t.v_max_out) {
    double mn = s_mn[lane], mx = s_mx[lane];
    for (int w = 1; w < kGW; ++w) {
      const double a = s_mn[w * 64 + lane], b = s_mx[w * 64 + lane];
      if (a == a) mn = (a < mn) ? a : mn;
      if (b == b) mx = (b > mx) ? b : mx;
    }
    if (t.v_min_out) t.v_min_out[e] = mn;
    if (t.v_max_out) t.v_max_out[e] = mx;
  }
  const int32_t itv = conv_ok ? my_it : -my_it;
  if (iters) iters[e] = itv;
  if (c.agent_power && c.coordinated) {
    const double v = s_vsel[lane];
    const double vv = pymax(pymax(0.0, c.vv_lo - v), v - c.vv_hi);
    if (c.vv) c.vv[e] = vv;
    const double share = (vv * c.vv_penalty) / (double)c.n_agents;
    // reward -= share (no-return atomic add of -share: one IEEE add per address)
#pragma unroll
    for (int ag = 0; ag < PGW_MAX_AGENTS; ++ag)
      if (ag < c.n_agents)
        (void)__hip_atomic_fetch_add(c.reward + (int64_t)ag * n + e, -share, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int CE, int CN>
static int32_t launch_general(const pgw_pfg_params& p, const pgw_pfg_tables& t, int64_t n, const double* cp,
                              const double* cq, double* v_out, int32_t* iters, const PFGCoord& c,
                              hipStream_t st) {
  if (p.n_reg > 0)
    launch_timed(PGW_T_PF_GENERAL, k_pf_general<CE, CN, true>, dim3((unsigned)((n + 63) / 64)), dim3(kBlock),
                 st, p, t, n, cp, cq, v_out, iters, c);
  else
    launch_timed(PGW_T_PF_GENERAL, k_pf_general<CE, CN, false>, dim3((unsigned)((n + 63) / 64)), dim3(kBlock),
                 st, p, t, n, cp, cq, v_out, iters, c);
  return check_launch("k_pf_general");
}

template <int CE>
static int32_t dispatch_cn(const pgw_pfg_params& p, const pgw_pfg_tables& t, int64_t n, const double* cp,
                           const double* cq, double* v_out, int32_t* iters, const PFGCoord& c, hipStream_t st) {
  if (p.mode == PGW_PF_EXACT) return launch_general<CE, 0>(p, t, n, cp, cq, v_out, iters, c, st);
  const int cn = (p.n_chk + 32 * 1 - 1) / 32;
  if (cn <= 1) return launch_general<CE, 1>(p, t, n, cp, cq, v_out, iters, c, st);
  if (cn <= 2) return launch_general<CE, 2>(p, t, n, cp, cq, v_out, iters, c, st);
  if (cn <= 4) return launch_general<CE, 4>(p, t, n, cp, cq, v_out, iters, c, st);
  return launch_general<CE, 8>(p, t, n, cp, cq, v_out, iters, c, st);
}

int32_t solve_general(const pgw_pfg_params* p, const pgw_pfg_tables* t, int64_t n, const double* cp,
                      const double* cq, double* v_out, int32_t* iters, const PFGCoord& c, void* stream) {
  PGW_REQUIRE(p && t && n >= 0, "pgw_pf_solve_general: null argument");
  PGW_REQUIRE(p->m >= 1 && p->m <= PGW_PFG_MAX_M && p->m % kGR == 0,
              "pgw_pf_solve_general: m=%d (need a multiple of 8, <= %d)", p->m, PGW_PFG_MAX_M);
  PGW_REQUIRE(t->elem && t->W && t->U0, "pgw_pf_solve_general: missing elem / W / U0");
  PGW_REQUIRE(p->mode == PGW_PF_EXACT || p->mode == PGW_PF_OPENDSS || p->mode == PGW_PF_OPENDSS_STEP,
              "pgw_pf_solve_general: bad mode");
  PGW_REQUIRE(p->mode == PGW_PF_EXACT ||
                  (p->n_chk >= kGR && p->n_chk <= PGW_PFG_MAX_CHK && p->n_chk % kGR == 0 && t->Gc && t->V0c),
              "pgw_pf_solve_general: OPENDSS needs n_chk check rows (multiple of 8, <= %d) and Gc / V0c",
              PGW_PFG_MAX_CHK);
  // (OPENDSS with U_init: OpenDSSSolver(snap_start="previous") -- each env's snap
  // solve starts from its previous solution instead of the direct one; the
  // stopping test counts from min_iter either way, so the check rows' first
  // magnitudes need no start value)
  PGW_REQUIRE(p->mode == PGW_PF_EXACT || !t->U_init || !p->n_reg,
              "pgw_pf_solve_general: OPENDSS with U_init and RegControls is not supported");
  PGW_REQUIRE(p->n_out >= 0 && (p->n_out == 0 || (t->G && t->V0)), "pgw_pf_solve_general: missing G / V0");
  PGW_REQUIRE(p->n_ctrl >= 0 && p->n_ctrl <= PGW_PF_MAX_CTRL, "pgw_pf_solve_general: bad n_ctrl");
  PGW_REQUIRE(p->max_iter >= 1 && p->min_iter >= 1, "pgw_pf_solve_general: bad iteration limits");
  PGW_REQUIRE(!c.agent_power || (c.vv_row >= 0 && c.vv_row < p->n_out),
              "pgw_pf_solve_general: bad coordinated voltage row");
  PGW_REQUIRE(p->n_reg >= 0 && p->n_reg <= PGW_PFG_MAX_REG && p->n_reg % kGR == 0 && p->r_reg >= 0 &&
                  p->r_reg <= p->n_reg && (p->n_reg == 0) == (p->r_reg == 0) &&
                  p->m + p->n_reg <= PGW_PFG_MAX_M,
              "pgw_pf_solve_general: bad n_reg %d / r_reg %d (m %d)", p->n_reg, p->r_reg, p->m);
  PGW_REQUIRE(p->n_reg == 0 || (t->Greg && t->V0reg && t->Kreg && t->reg_x && t->reg_c && t->reg_rho),
              "pgw_pf_solve_general: regulators need Greg / V0reg / Kreg / reg_x / reg_c / reg_rho");
  PGW_REQUIRE(p->n_reg == 0 || !c.agent_power, "pgw_pf_solve_general: regulators on the fused step");
  if (n == 0) return PGW_OK;
  hipStream_t st = (hipStream_t)stream;
  const int cols = p->m + p->n_reg;
  if (cols <= 32) return dispatch_cn<1>(*p, *t, n, cp, cq, v_out, iters, c, st);
  if (cols <= 64) return dispatch_cn<2>(*p, *t, n, cp, cq, v_out, iters, c, st);
  return dispatch_cn<4>(*p, *t, n, cp, cq, v_out, iters, c, st);
}

}  // namespace pgw

using namespace pgw;

extern "C" {

int32_t pgw_pf_solve_general(const pgw_pfg_params* p, const pgw_pfg_tables* t, int64_t n,
                             const double* ctrl_p, const double* ctrl_q, double* v_out, int32_t* iters,
                             void* stream) {
  const PFGCoord c = {};
  return solve_general(p, t, n, ctrl_p, ctrl_q, v_out, iters, c, stream);
}

}  // extern "C"
