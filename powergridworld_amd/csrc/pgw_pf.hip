// Batched distribution power flow + the coordinated multi-building step.
//
// Power flow (replaces the OpenDSS snap solve behind opendss.py:80-165): per env,
// fixed-point current injection on the m load-element voltages
//     U <- U0 + W f(U),   f = OpenDSS PQ-load current law (model 1),
// with W = -C Z C^T, U0 = C V0 precomputed on the host (pgw_feeder.cpp) and
// shared by every env.  One thread per env keeps its U, I and element powers
// in registers; everything shared (W, U0, the output rows of G, per-element
// thresholds) is staged ONCE per workgroup in LDS and read as wave-uniform
// broadcasts, so the inner loop is fp64 FMAs + broadcast ds_reads.
//
// Coordinated step (the BASELINE C4 path) = two launches on one stream:
//   k_coord_agents  one thread per (env, agent): building + PV + storage step,
//                   obs/state writes, agent real power and (pre-transform) reward
//                   -- pure HBM streaming, 5x the waves of a per-env kernel;
//   k_coord_pf      one thread per env: bus loads = sum of agent powers, power
//                   flow, voltage-violation penalty folded into the rewards.
#include <algorithm>

#include "pgw_common.h"

namespace pgw {

constexpr int kMaxOutLds = 48;   // output rows staged in LDS (IEEE-13 has 38 nodes)

// ----------------------------------------------------------------------------
// MFMA layout (v_mfma_f64_16x16x4f64, decoded on gfx950 by
// tools/micro/mfma_f64_layout.hip): A lane l holds A[l%16][l/16], B lane l holds
// B[l/16][l%16], and D lane l holds D[4r + l/16][l%16] for r = 0..3.
//
// A wave solves 16 envs: env = lane % 16, sub-lane q = lane / 16.  Element k
// (padded to 16) is owned by sub-lane q = k % 4 in slot r = k / 4.  In real form
//     [Ur; Ui] = U0 + [[Wre, -Wim], [Wim, Wre]] [Ir; Ii]      (32 x 32)
// the B operand of k-step s is x[4s + q] -- the lane's OWN current (slot s % 4,
// real part for s < 4, imaginary part otherwise) -- and D row 4r + q of row
// block rb is the real (rb 0) / imaginary (rb 1) part of the lane's OWN element
// 4r + q.  So one iteration = currents on the VALU + 16 MFMAs on the matrix
// pipe, with no cross-lane data movement at all; W lives in 16 f64 registers
// per lane for the whole solve.
// ----------------------------------------------------------------------------
typedef double pgw_double4 __attribute__((ext_vector_type(4)));

constexpr int kPfElem = 16;       // padded element count of the MFMA layout

struct PFShared {
  double2 U0[kPfElem];
  double4 thr[kPfElem];            // (lo^2, mn^2, mx^2, 1/vb^2) in V^2
  double4 gsc[kPfElem];            // (g_low, g_min, g_max, -)
  double2 G[kMaxOutLds * kPfElem];
  double2 V0[kMaxOutLds];
  double inv_vbase_out[kMaxOutLds];
  double2 Upred[3][kPfElem];       // predictor solutions (if any)
};

// Cooperative staging of the shared PF tables (all threads of the block).
// Tables from the host are J x J (W), J (U0), n_out x J (G) with J <= 16.
__device__ __forceinline__ void pf_stage(PFShared& S, const pgw_pf_params& p,
                                         const pgw_pf_tables& t, int J, int n_out_lds) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const double2* U0 = reinterpret_cast<const double2*>(t.U0);
  for (int i = tid; i < kPfElem; i += nt) {
    const bool real = i < J;
    S.U0[i] = real ? U0[i] : make_double2(0.0, 0.0);
    const double vb = real ? p.vbase[i] : 1.0;
    const double vmin = real ? p.vmin[i] : 0.95, vmax = real ? p.vmax[i] : 1.05;
    const double vlow = real ? p.vlow[i] : 0.5;
    const double vb2 = vb * vb;
    const double lo = vlow * vb, mn = vmin * vb, mx = vmax * vb;
    S.thr[i] = make_double4(lo * lo, mn * mn, mx * mx, 1.0 / vb2);
    S.gsc[i] = make_double4(1.0 / vb2, 1.0 / (vb2 * (vmin * vmin)), 1.0 / (vb2 * (vmax * vmax)), 0.0);
  }
  const double2* G = reinterpret_cast<const double2*>(t.G);
  for (int i = tid; i < n_out_lds * kPfElem; i += nt) {
    const int o = i / kPfElem, k = i % kPfElem;
    S.G[i] = (k < J) ? G[o * J + k] : make_double2(0.0, 0.0);
  }
  const double2* V0 = reinterpret_cast<const double2*>(t.V0);
  for (int i = tid; i < n_out_lds; i += nt) {
    S.V0[i] = V0[i];
    S.inv_vbase_out[i] = t.inv_vbase_out[i];
  }
  if (t.U_pred) {
    const double2* Up = reinterpret_cast<const double2*>(t.U_pred);
    for (int i = tid; i < 3 * kPfElem; i += nt) {
      const int c = i / kPfElem, k = i % kPfElem;
      S.Upred[c][k] = (k < J) ? Up[c * J + k] : make_double2(0.0, 0.0);
    }
  }
}

__device__ __forceinline__ double fast_rcp(double m) {
  // v_rcp_f64 + two Newton steps (~1 ulp; the exact IEEE divide sequence costs
  // ~3x more and the PF is iterated to a tolerance anyway)
  double r = __builtin_amdgcn_rcp(m);
  double e = fma(-m, r, 1.0);
  r = fma(r, e, r);
  e = fma(-m, r, 1.0);
  return fma(r, e, r);
}

// Reductions over the 4 sub-lanes of an env (lanes n, n+16, n+32, n+48).
__device__ __forceinline__ double sub_max(double v) {
  double o = __shfl_xor(v, 16);
  v = (o > v) ? o : v;
  o = __shfl_xor(v, 32);
  return (o > v) ? o : v;
}
__device__ __forceinline__ double sub_sum(double v) {
  v = v + __shfl_xor(v, 16);
  return v + __shfl_xor(v, 32);
}

// OpenDSS Load.DoConstantPQLoad: every case is I = conj(S) U g with
//   g = 1/|U|^2 (constant PQ, vmin < |U|/vb <= vmax) or the constant-Z scale
//   1/(vb vmin)^2 (below vmin), 1/(vb vmax)^2 (above vmax), 1/vb^2 (below vlow).
__device__ __forceinline__ void pf_current(const double4& th, const double4& gs, double sw,
                                           double sv, double ur, double ui, double& ir,
                                           double& ii) {
  const double m2 = ur * ur + ui * ui;
  double g = fast_rcp(m2);
  g = (m2 > th.z) ? gs.z : g;
  g = (m2 <= th.y) ? gs.y : g;
  g = (m2 <= th.x) ? gs.x : g;
  ir = (sw * ur + sv * ui) * g;
  ii = (sw * ui - sv * ur) * g;
}

// Per-lane state: the lane's 4 owned elements k = 4r + q.
struct PFLane {
  double sw[4], sv[4];        // element powers (W, var)
  double ur[4], ui[4];        // element voltages
  double ir[4], ii[4];        // element currents
};

// The lane's 16 A operands: A[rb][s] = Wreal[16 rb + (l%16)][4 s + q].
struct PFMatrix {
  double a[2][8];
};

__device__ __forceinline__ void pf_load_matrix(const pgw_pf_tables& t, int J, int lane,
                                               PFMatrix& Mx) {
  const int i = lane & 15, q = lane >> 4;
  const double2* W = reinterpret_cast<const double2*>(t.W);
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int c = 4 * (s & 3) + q;           // element column
    const bool imag_col = s >= 4;            // x = Ii for k-steps 4..7
    double wre = 0.0, wim = 0.0;
    if (i < J && c < J) {
      const double2 w = W[i * J + c];
      wre = w.x;
      wim = w.y;
    }
    // rb 0 (real rows): Wre Ir - Wim Ii ;  rb 1 (imag rows): Wim Ir + Wre Ii
    Mx.a[0][s] = imag_col ? -wim : wre;
    Mx.a[1][s] = imag_col ? wre : wim;
  }
}

__device__ __forceinline__ void pf_own_currents(const PFShared& S, int q, PFLane& L) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int k = 4 * r + q;
    pf_current(S.thr[k], S.gsc[k], L.sw[r], L.sv[r], L.ur[r], L.ui[r], L.ir[r], L.ii[r]);
  }
}

// Fixed-point solve for the wave's 16 envs.  Every lane of a wave stays in the
// loop (the MFMAs need the full wave) until all 16 envs have converged; an env
// that converged keeps its voltages (frozen), so each env's result and
// iteration count are those of iterating it alone.
__device__ __forceinline__ int pf_solve(const PFShared& S, const PFMatrix& Mx,
                                        const pgw_pf_params& p, int q, bool valid, PFLane& L,
                                        bool pred, double pc) {
  if (pred) {
    // quadratic Lagrange interpolation of the 3 reference solutions at pc
    const double x0 = p.pred_p[0], x1 = p.pred_p[1], x2 = p.pred_p[2];
    const double w0 = ((pc - x1) * (pc - x2)) / ((x0 - x1) * (x0 - x2));
    const double w1 = ((pc - x0) * (pc - x2)) / ((x1 - x0) * (x1 - x2));
    const double w2 = ((pc - x0) * (pc - x1)) / ((x2 - x0) * (x2 - x1));
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = 4 * r + q;
      L.ur[r] = w0 * S.Upred[0][k].x + w1 * S.Upred[1][k].x + w2 * S.Upred[2][k].x;
      L.ui[r] = w0 * S.Upred[0][k].y + w1 * S.Upred[1][k].y + w2 * S.Upred[2][k].y;
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      L.ur[r] = S.U0[4 * r + q].x;
      L.ui[r] = S.U0[4 * r + q].y;
    }
  }
  const double tol2 = p.tol * p.tol;
  int it = 0, my_it = 0;
  bool done = !valid;
  while (it < p.max_iter) {
    ++it;
    asm volatile("" ::: "memory");
    pf_own_currents(S, q, L);
    pgw_double4 acc0, acc1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      acc0[r] = S.U0[4 * r + q].x;
      acc1[r] = S.U0[4 * r + q].y;
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const double b = (s < 4) ? L.ir[s & 3] : L.ii[s & 3];
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(Mx.a[0][s], b, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(Mx.a[1][s], b, acc1, 0, 0, 0);
    }
    double err2 = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = 4 * r + q;
      const double dr = acc0[r] - L.ur[r], di = acc1[r] - L.ui[r];
      const double e2 = (dr * dr + di * di) * S.thr[k].w;
      err2 = (e2 > err2) ? e2 : err2;
      L.ur[r] = done ? L.ur[r] : acc0[r];
      L.ui[r] = done ? L.ui[r] : acc1[r];
    }
    err2 = sub_max(err2);
    if (!done) {
      my_it = it;
      done = err2 < tol2;
    }
    if (__ballot(!done) == 0ull) break;
  }
  pf_own_currents(S, q, L);
  return valid ? (done ? my_it : it) : 0;
}

// |V| pu of output row o: V0 + sum_k G[o][k] I_k -- each sub-lane sums its own
// elements, then a sum over the 4 sub-lanes (every lane returns the value).
__device__ __forceinline__ double pf_node_pu(const PFShared& S, const pgw_pf_tables& t, int J,
                                             int o, int q, const PFLane& L) {
  double vr = 0.0, vi = 0.0;
  const bool lds = o < kMaxOutLds;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int k = 4 * r + q;
    double gx = 0.0, gy = 0.0;
    if (lds) {
      gx = S.G[o * kPfElem + k].x;
      gy = S.G[o * kPfElem + k].y;
    } else if (k < J) {
      gx = t.G[2 * (o * J + k)];
      gy = t.G[2 * (o * J + k) + 1];
    }
    vr = fma(gx, L.ir[r], vr);
    vr = fma(-gy, L.ii[r], vr);
    vi = fma(gx, L.ii[r], vi);
    vi = fma(gy, L.ir[r], vi);
  }
  vr = sub_sum(vr);
  vi = sub_sum(vi);
  const double v0r = lds ? S.V0[o].x : t.V0[2 * o], v0i = lds ? S.V0[o].y : t.V0[2 * o + 1];
  vr = v0r + vr;
  vi = v0i + vi;
  return sqrt(vr * vr + vi * vi) * (lds ? S.inv_vbase_out[o] : t.inv_vbase_out[o]);
}

__device__ __forceinline__ void pf_store_u(const pgw_pf_tables& t, int J, int64_t e, int q,
                                           const PFLane& L) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int k = 4 * r + q;
    if (k < J) {
      t.U_out[2 * (e * J + k)] = L.ur[r];
      t.U_out[2 * (e * J + k) + 1] = L.ui[r];
    }
  }
}

// Own element powers (opendss.py:107-129; OpenDSS WNominal = kW*1000/nphases).
__device__ __forceinline__ void pf_element_powers(const pgw_pf_params& p, int J, const double* cp,
                                                  const double* cq, int q, PFLane& L) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int k = 4 * r + q;
    double sw = 0.0, sv = 0.0;
    if (k < J) {
      double kw = p.base_kw[k], kvar = p.base_kvar[k];
      const int c = p.elem_ctrl[k];
      if (c >= 0) {
        double pc = cp[0], qc = cq[0];
#pragma unroll
        for (int s = 1; s < PGW_PF_MAX_CTRL; ++s) {
          pc = (c == s) ? cp[s] : pc;
          qc = (c == s) ? cq[s] : qc;
        }
        kw = kw + pc;
        kvar = kvar + qc;
      }
      sw = (kw * 1000.0) / p.nph[k];
      sv = (kvar * 1000.0) / p.nph[k];
    }
    L.sw[r] = sw;
    L.sv[r] = sv;
  }
}

constexpr int kEnvsPerBlock = kBlock / 4;   // 16 envs per wave

__device__ __forceinline__ int64_t pf_env_index(int lane) {
  return (int64_t)blockIdx.x * kEnvsPerBlock + (threadIdx.x >> 6) * 16 + (lane & 15);
}

__global__ void __launch_bounds__(kBlock) k_pf_solve(pgw_pf_params p, pgw_pf_tables t, int64_t n,
                                                     const double* __restrict__ ctrl_p,
                                                     const double* __restrict__ ctrl_q,
                                                     double* __restrict__ v_out,
                                                     int32_t* __restrict__ iters) {
  __shared__ PFShared S;
  const int J = p.m;
  const int n_lds = p.n_out < kMaxOutLds ? p.n_out : kMaxOutLds;
  pf_stage(S, p, t, J, n_lds);
  const int lane = threadIdx.x & 63, q = lane >> 4;
  PFMatrix Mx;
  pf_load_matrix(t, J, lane, Mx);
  __syncthreads();
  const int64_t e = pf_env_index(lane);
  const bool valid = e < n;
  if (__ballot(valid) == 0ull) return;      // whole wave out of range
  double cp[PGW_PF_MAX_CTRL], cq[PGW_PF_MAX_CTRL];
#pragma unroll
  for (int c = 0; c < PGW_PF_MAX_CTRL; ++c) {
    cp[c] = (valid && c < p.n_ctrl && ctrl_p) ? ctrl_p[(int64_t)c * n + e] : 0.0;
    cq[c] = (valid && c < p.n_ctrl && ctrl_q) ? ctrl_q[(int64_t)c * n + e] : 0.0;
  }
  PFLane L;
  pf_element_powers(p, J, cp, cq, q, L);
  const int it = pf_solve(S, Mx, p, q, valid, L, t.U_pred != nullptr && p.n_ctrl == 1, cp[0]);
  for (int o = 0; o < p.n_out; ++o) {
    const double v = pf_node_pu(S, t, J, o, q, L);
    if (valid && q == 0) v_out[(int64_t)o * n + e] = v;
  }
  if (valid && t.U_out) pf_store_u(t, J, e, q, L);
  if (valid && iters && q == 0) iters[e] = it;
}

// ============================================================ coordinated step
// K1: one thread per (env, agent) -- MultiComponentEnv.step (base.py:114-139) of
// one [building, pv, storage] agent (scenarios/buildings.py:11-72) with the
// fresh reward (base.py:137): 0. + building + pv(0) + storage(0).
__global__ void __launch_bounds__(kBlock) k_coord_agents(pgw_coord_params p, pgw_coord_step_info s,
                                                         int64_t n, pgw_coord_buffers b) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int a = blockIdx.y;
  if (e >= n) return;
  pgw_mat act = b.action;
  act.ptr += a * b.act_stride_agent;
  pgw_mat obs = b.obs;
  obs.ptr += a * b.obs_stride_agent;
  double agent_rp = 0.0, r_bld = 0.0;
  for (int ci = 0; ci < p.n_comp; ++ci) {
    const int comp = p.comp_order[ci];
    if (comp == 0) {
      // building: five_zone_rom_env.py:183-225
      double av[6], xs[5], T[5];
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const double v = ld(act, e, p.act_bld + j);
        av[j] = p.bld.rescale ? to_raw(v, p.bld.act_low[j], p.bld.act_high[j]) : v;
      }
      double* xp = b.x + (int64_t)a * 5 * n;
#pragma unroll
      for (int z = 0; z < 5; ++z) {
        xs[z] = xp[z * n + e];
        T[z] = p.bld.C[z] * xs[z] + p.bld.mean[z];
      }
      building_state_update(p.bld, s.ex_t, T, av, xs);
#pragma unroll
      for (int z = 0; z < 5; ++z) {
        xp[z * n + e] = xs[z];
        T[z] = p.bld.C[z] * xs[z] + p.bld.mean[z];
      }
      const double pc = building_p_consumed(av, s.ex_t.T_oa);
      r_bld = building_reward(p.bld, T, s.ex_next.comfort_lb, s.ex_next.comfort_ub, pc);
      const BuildingExt xv = {1.0, 1.0, 1.0, __builtin_huge_val()};
      building_write_obs(p.bld, T, s.ex_next, pc, xv,
                         [&](int j, double v) { st(obs, e, p.obs_bld + j, v); });
      agent_rp = agent_rp + pc;
    } else if (comp == 1) {
      // PV: pv_profile_env.py:133-148
      st(obs, e, p.obs_pv, pv_obs(p.pv, s.pv_pmax));
      agent_rp = agent_rp + pv_real_power(p.pv, ld(act, e, p.act_pv), s.pv_pmax);
    } else {
      // storage: energy_storage_env.py:131-157
      double soc = b.soc[(int64_t)a * n + e];
      const double power = battery_step(p.bat, ld(act, e, p.act_bat), soc);
      b.soc[(int64_t)a * n + e] = soc;
      st(obs, e, p.obs_bat, battery_obs(p.bat, soc));
      agent_rp = agent_rp + (-power);
    }
  }
  double agent_rew = 0.0;
  for (int ci = 0; ci < p.n_comp; ++ci) agent_rew = agent_rew + (p.comp_order[ci] == 0 ? r_bld : 0.0);
  b.agent_power[(int64_t)a * n + e] = agent_rp;
  b.reward[(int64_t)a * n + e] = agent_rew;
}

// K1 fast path: the standard C4 agent -- components [building, pv, storage]
// at action offsets 0/6/7, the reference's 5-zone model structure
// (input_sel_list [1,8,x,2], state_space_model.p) and the default building
// observation config (defaults.py:2-10).  Same arithmetic, operation for
// operation, as the generic device functions (the fused-vs-generic test checks
// bit equality); only the uniform selects become compile-time indices.

__global__ void __launch_bounds__(kBlock) k_coord_agents_std(pgw_coord_params p,
                                                             pgw_coord_step_info s, int64_t n,
                                                             pgw_coord_buffers b, double pv_ob) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int a = blockIdx.y;
  if (e >= n) return;
  const pgw_building_params& B = p.bld;
  const double* ap = b.action.ptr + a * b.act_stride_agent + e * b.action.s_env;
  const int64_t sd = b.action.s_dim;
  double av[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) av[j] = ap[j * sd];
  double* xp = b.x + (int64_t)a * 5 * n + e;
  double xs[5], T[5];
#pragma unroll
  for (int z = 0; z < 5; ++z) xs[z] = xp[z * n];
  // ---- building
#pragma unroll
  for (int j = 0; j < 6; ++j) av[j] = B.rescale ? to_raw(av[j], B.act_low[j], B.act_high[j]) : av[j];
#pragma unroll
  for (int z = 0; z < 5; ++z) T[z] = B.C[z] * xs[z] + B.mean[z];
  double nb[5];
  nb[0] = T[4]; nb[1] = T[4]; nb[2] = T[3]; nb[3] = T[2]; nb[4] = T[2];
#pragma unroll
  for (int z = 0; z < 5; ++z) {
    const double u0 = s.ex_t.T_oa - T[z];
    const double u1 = av[z] * (av[5] - T[z]);
    const double u2 = nb[z] - T[z];
    const double u3 = s.ex_t.q_solar[z];
    double bu = B.B[z][0] * u0;
    bu = bu + B.B[z][1] * u1;
    bu = bu + B.B[z][2] * u2;
    bu = bu + B.B[z][3] * u3;
    xs[z] = B.A[z] * xs[z] + bu;
  }
#pragma unroll
  for (int z = 0; z < 5; ++z) {
    xp[z * n] = xs[z];
    T[z] = B.C[z] * xs[z] + B.mean[z];
  }
  const double pc = building_p_consumed(av, s.ex_t.T_oa);
  const double lb = s.ex_next.comfort_lb, ub = s.ex_next.comfort_ub;
  const double r_bld = building_reward(B, T, lb, ub, pc);
  double* op = b.obs.ptr + a * b.obs_stride_agent + e * b.obs.s_env;
  const int64_t so = b.obs.s_dim;
  double ov[15];
#pragma unroll
  for (int z = 0; z < 5; ++z) {
    ov[z] = T[z] - ub;
    ov[5 + z] = lb - T[z];
  }
  ov[10] = lb;
  ov[11] = ub;
  ov[12] = s.ex_next.T_oa;
  ov[13] = pc;
  ov[14] = s.ex_next.time_of_day;
#pragma unroll
  for (int j = 0; j < 15; ++j) {
    double v = clip(ov[j], B.obs_low[j], B.obs_high[j]);
    if (B.rescale) v = to_scaled(v, B.obs_low[j], B.obs_high[j]);
    op[j * so] = v;
  }
  // ---- pv (obs is env-independent: computed once on the host)
  op[15 * so] = pv_ob;
  const double rp_pv = pv_real_power(p.pv, av[6], s.pv_pmax);
  // ---- storage
  double* socp = b.soc + (int64_t)a * n + e;
  double soc = *socp;
  const double power = battery_step(p.bat, av[7], soc);
  *socp = soc;
  op[16 * so] = battery_obs(p.bat, soc);
  // MultiComponentEnv sums (base.py:131-137)
  double agent_rp = 0.0;
  agent_rp = agent_rp + pc;
  agent_rp = agent_rp + rp_pv;
  agent_rp = agent_rp + (-power);
  double agent_rew = 0.0;
  agent_rew = agent_rew + r_bld;
  agent_rew = agent_rew + 0.0;
  agent_rew = agent_rew + 0.0;
  b.agent_power[(int64_t)a * n + e] = agent_rp;
  b.reward[(int64_t)a * n + e] = agent_rew;
}

static bool coord_is_std(const pgw_coord_params& p) {
  static const int sel[5][4] = {{0, 7, 6, 1}, {0, 7, 6, 1}, {0, 7, 5, 1}, {0, 7, 5, 1}, {0, 7, 5, 1}};
  static const int nbr[5][4] = {{1, 2, 3, 4}, {0, 2, 3, 4}, {0, 1, 3, 4}, {0, 1, 2, 4}, {0, 1, 2, 3}};
  if (p.n_comp != 3 || p.comp_order[0] != 0 || p.comp_order[1] != 1 || p.comp_order[2] != 2)
    return false;
  if (p.act_bld != 0 || p.act_pv != 6 || p.act_bat != 7 || p.act_dim != 8) return false;
  if (p.obs_bld != 0 || p.obs_pv != 15 || p.obs_bat != 16 || p.obs_dim != 17) return false;
  if (p.pv.grid_aware || p.bld.n_obs != 15) return false;
  for (int z = 0; z < 5; ++z)
    for (int j = 0; j < 4; ++j)
      if (p.bld.sel[z][j] != sel[z][j] || p.bld.nbr[z][j] != nbr[z][j]) return false;
  for (int j = 0; j < 15; ++j)
    if (p.bld.obs_var[j] != 5 + j) return false;
  return true;
}

// K2: 4 lanes per env (MFMA layout above) -- bus loads (multiagent_env.py:171-181),
// power flow (opendss.py:80-135), CoordinatedMultiBuildingControlEnv.reward_transform
// (train.py:51-63, 71-88) applied to the agent rewards in place.
__global__ void __launch_bounds__(kBlock) k_coord_pf(pgw_coord_params p, pgw_pf_params pf,
                                                     pgw_pf_tables pft, int64_t n,
                                                     pgw_coord_buffers b) {
  __shared__ PFShared S;
  const int J = pf.m;
  const int n_lds = pf.n_out < kMaxOutLds ? pf.n_out : kMaxOutLds;
  pf_stage(S, pf, pft, J, n_lds);
  const int lane = threadIdx.x & 63, q = lane >> 4;
  PFMatrix Mx;
  pf_load_matrix(pft, J, lane, Mx);
  __syncthreads();
  const int64_t e = pf_env_index(lane);
  const bool valid = e < n;
  if (__ballot(valid) == 0ull) return;
  double cp[PGW_PF_MAX_CTRL], cq[PGW_PF_MAX_CTRL];
#pragma unroll
  for (int c = 0; c < PGW_PF_MAX_CTRL; ++c) {
    cp[c] = 0.0;
    cq[c] = 0.0;
  }
  if (valid) {
    for (int a = 0; a < p.n_agents; ++a) {
      const double rp = b.agent_power[(int64_t)a * n + e];
      const int slot = p.agent_ctrl[a];
#pragma unroll
      for (int c = 0; c < PGW_PF_MAX_CTRL; ++c) cp[c] = (c == slot) ? cp[c] + rp : cp[c];
    }
  }
  PFLane L;
  pf_element_powers(pf, J, cp, cq, q, L);
  const int it = pf_solve(S, Mx, pf, q, valid, L, pft.U_pred != nullptr && pf.n_ctrl == 1, cp[0]);
  double vsel = 0.0;
  for (int o = 0; o < pf.n_out; ++o) {
    const double v = pf_node_pu(S, pft, J, o, q, L);
    if (valid && b.v_out && q == 0) b.v_out[(int64_t)o * n + e] = v;
    vsel = (o == p.vv_row) ? v : vsel;
  }
  if (!valid) return;
  if (b.iters && q == 0) b.iters[e] = it;
  if (p.coordinated) {
    const double vv = pymax(pymax(0.0, p.vv_lo - vsel), vsel - p.vv_hi);
    if (b.vv && q == 0) b.vv[e] = vv;
    const double share = (vv * p.vv_penalty) / (double)p.n_agents;
    for (int a = q; a < p.n_agents; a += 4) {
      double* r = b.reward + (int64_t)a * n + e;
      *r = *r - share;
    }
  }
}

// padded element count actually used by the device tables for a given m
// (the MFMA layout pads to 16 internally; host tables are m x m, m <= 16)
static int padded_m(int m) { return m; }

}  // namespace pgw

using namespace pgw;

extern "C" {

int32_t pgw_pf_padded_m(int32_t m) { return padded_m(m); }

int32_t pgw_pf_solve(const pgw_pf_params* p, const pgw_pf_tables* t, int64_t n,
                     const double* ctrl_p, const double* ctrl_q, double* v_out, int32_t* iters,
                     void* stream) {
  PGW_REQUIRE(p && t && t->W && t->U0 && v_out && n >= 0, "pgw_pf_solve: null argument");
  PGW_REQUIRE(p->m >= 1 && p->m <= PGW_PF_MAX_M && p->m == padded_m(p->m),
              "pgw_pf_solve: m=%d out of range", p->m);
  PGW_REQUIRE(p->n_ctrl >= 0 && p->n_ctrl <= PGW_PF_MAX_CTRL, "pgw_pf_solve: bad n_ctrl");
  PGW_REQUIRE(p->n_out == 0 || (t->G && t->V0 && t->inv_vbase_out), "pgw_pf_solve: missing G/V0");
  PGW_REQUIRE(p->max_iter >= 1, "pgw_pf_solve: max_iter < 1");
  if (n == 0) return PGW_OK;
  hipLaunchKernelGGL(k_pf_solve, dim3(grid_for(4 * n)), dim3(kBlock), 0, (hipStream_t)stream, *p,
                     *t, n, ctrl_p, ctrl_q, v_out, iters);
  return check_launch("k_pf_solve");
}

int32_t pgw_coord_step(const pgw_coord_params* p, const pgw_pf_params* pf, const pgw_pf_tables* pft,
                       const pgw_coord_step_info* s, int64_t n, pgw_coord_buffers b, void* stream) {
  PGW_REQUIRE(p && pf && pft && s && n >= 0, "pgw_coord_step: null argument");
  PGW_REQUIRE(p->n_agents >= 1 && p->n_agents <= PGW_MAX_AGENTS, "pgw_coord_step: bad n_agents");
  PGW_REQUIRE(p->n_comp >= 1 && p->n_comp <= 3, "pgw_coord_step: bad n_comp");
  PGW_REQUIRE(b.action.ptr && b.obs.ptr && b.reward && b.agent_power,
              "pgw_coord_step: null buffer");
  PGW_REQUIRE(pf->m >= 1 && pf->m <= PGW_PF_MAX_M && pf->m == padded_m(pf->m),
              "pgw_coord_step: pf m=%d not padded", pf->m);
  PGW_REQUIRE(pf->n_out >= 1 && p->vv_row >= 0 && p->vv_row < pf->n_out,
              "pgw_coord_step: bad vv_row");
  PGW_REQUIRE(pf->max_iter >= 1, "pgw_coord_step: max_iter < 1");
  for (int a = 0; a < p->n_agents; ++a)
    PGW_REQUIRE(p->agent_ctrl[a] < pf->n_ctrl, "pgw_coord_step: agent_ctrl out of range");
  for (int c = 0; c < p->n_comp; ++c) {
    int k = p->comp_order[c];
    PGW_REQUIRE(k >= 0 && k <= 2, "pgw_coord_step: bad comp_order");
    if (k == 0) PGW_REQUIRE(b.x && p->act_bld >= 0 && p->bld.n_obs <= PGW_BLD_MAX_OBS, "pgw_coord_step: building");
    if (k == 2) PGW_REQUIRE(b.soc && p->act_bat >= 0, "pgw_coord_step: storage");
  }
  if (n == 0) return PGW_OK;
  hipStream_t st = (hipStream_t)stream;
  if (coord_is_std(*p)) {
    // PVEnv.get_obs is the same for every env: evaluate it once here
    const double pv_ob = p->pv.rescale ? (2.0 * std::min(std::max(-s->pv_pmax, p->pv.obs_low), p->pv.obs_high)
                                          - (p->pv.obs_low + p->pv.obs_high)) / (p->pv.obs_high - p->pv.obs_low)
                                       : -s->pv_pmax;
    hipLaunchKernelGGL(k_coord_agents_std, dim3(grid_for(n), p->n_agents), dim3(kBlock), 0, st, *p,
                       *s, n, b, pv_ob);
  } else {
    hipLaunchKernelGGL(k_coord_agents, dim3(grid_for(n), p->n_agents), dim3(kBlock), 0, st, *p, *s,
                       n, b);
  }
  int32_t rc = check_launch("k_coord_agents");
  if (rc) return rc;
  hipLaunchKernelGGL(k_coord_pf, dim3(grid_for(4 * n)), dim3(kBlock), 0, st, *p, *pf, *pft, n, b);
  return check_launch("k_coord_pf");
}

}  // extern "C"
