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
// Quad layout: the 4 consecutive lanes q = lane & 3 of a quad solve ONE env.
// Element k is owned by lane k & 3 (slot r = k >> 2): that lane holds U_k, the
// element power and computes I_k and row k of the matvec.  Each iteration the
// J currents are exchanged inside the quad with DPP quad_perm broadcasts, so
// the per-env work is split four ways with no LDS traffic for per-env data:
// 4x the waves of a one-lane-per-env solver (latency hiding at 1 wave/SIMD was
// the bottleneck), identical arithmetic per row.
// ----------------------------------------------------------------------------
template <int J>
struct QuadDims {
  static constexpr int R = (J + 3) / 4;   // element slots per lane
  static constexpr int K = 4 * R;         // padded row count
};

template <int J>
struct PFShared {
  double2 W[QuadDims<J>::K * J];          // rows padded to K with zeros
  double2 U0[QuadDims<J>::K];
  double4 thr[QuadDims<J>::K];            // (lo^2, mn^2, mx^2, 1/vb^2) in V^2
  double4 gsc[QuadDims<J>::K];            // (g_low, g_min, g_max, -)
  double2 G[kMaxOutLds * J];
  double2 V0[kMaxOutLds];
  double inv_vbase_out[kMaxOutLds];
  double2 Upred[3][QuadDims<J>::K];       // predictor solutions (if any)
};

// Cooperative staging of the shared PF tables (all threads of the block).
template <int J>
__device__ __forceinline__ void pf_stage(PFShared<J>& S, const pgw_pf_params& p,
                                         const pgw_pf_tables& t, int n_out_lds) {
  constexpr int K = QuadDims<J>::K;
  const int tid = threadIdx.x, nt = blockDim.x;
  const double2* W = reinterpret_cast<const double2*>(t.W);
  for (int i = tid; i < K * J; i += nt) S.W[i] = (i < J * J) ? W[i] : make_double2(0.0, 0.0);
  const double2* U0 = reinterpret_cast<const double2*>(t.U0);
  for (int i = tid; i < K; i += nt) {
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
  for (int i = tid; i < n_out_lds * J; i += nt) S.G[i] = G[i];
  const double2* V0 = reinterpret_cast<const double2*>(t.V0);
  for (int i = tid; i < n_out_lds; i += nt) {
    S.V0[i] = V0[i];
    S.inv_vbase_out[i] = t.inv_vbase_out[i];
  }
  if (t.U_pred) {
    const double2* Up = reinterpret_cast<const double2*>(t.U_pred);
    for (int i = tid; i < 3 * K; i += nt) {
      const int c = i / K, k = i % K;
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

// DPP quad_perm on a double (two 32-bit moves).  CTRL = quad_perm selector.
template <int CTRL>
__device__ __forceinline__ double dpp_quad(double v) {
  unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  int lo = __builtin_amdgcn_mov_dpp((int)(u & 0xffffffffull), CTRL, 0xF, 0xF, false);
  int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), CTRL, 0xF, 0xF, false);
  unsigned long long w = ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
  return __builtin_bit_cast(double, w);
}
template <int S>
__device__ __forceinline__ double quad_bcast(double v) { return dpp_quad<S * 0x55>(v); }
__device__ __forceinline__ double quad_max(double v) {
  double o = dpp_quad<0xB1>(v);      // [1,0,3,2]
  v = (o > v) ? o : v;
  o = dpp_quad<0x4E>(v);             // [2,3,0,1]
  return (o > v) ? o : v;
}
__device__ __forceinline__ double quad_sum(double v) {
  v = v + dpp_quad<0xB1>(v);
  return v + dpp_quad<0x4E>(v);
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

// Per-lane state of one quad lane.
template <int J>
struct PFLane {
  static constexpr int R = QuadDims<J>::R;
  double sw[R], sv[R];        // own element powers (W, var)
  double ur[R], ui[R];        // own element voltages
  double ir[R], ii[R];        // own element currents
};

// All J currents of the env, gathered from the quad.
template <int J>
__device__ __forceinline__ void quad_gather(const PFLane<J>& L, double Ir[J], double Ii[J]) {
  constexpr int R = QuadDims<J>::R;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (4 * r + 0 < J) { Ir[4 * r + 0] = quad_bcast<0>(L.ir[r]); Ii[4 * r + 0] = quad_bcast<0>(L.ii[r]); }
    if (4 * r + 1 < J) { Ir[4 * r + 1] = quad_bcast<1>(L.ir[r]); Ii[4 * r + 1] = quad_bcast<1>(L.ii[r]); }
    if (4 * r + 2 < J) { Ir[4 * r + 2] = quad_bcast<2>(L.ir[r]); Ii[4 * r + 2] = quad_bcast<2>(L.ii[r]); }
    if (4 * r + 3 < J) { Ir[4 * r + 3] = quad_bcast<3>(L.ir[r]); Ii[4 * r + 3] = quad_bcast<3>(L.ii[r]); }
  }
}

template <int J>
__device__ __forceinline__ void pf_own_currents(const PFShared<J>& S, int q, PFLane<J>& L) {
#pragma unroll
  for (int r = 0; r < QuadDims<J>::R; ++r) {
    const int k = 4 * r + q;
    pf_current(S.thr[k], S.gsc[k], L.sw[r], L.sv[r], L.ur[r], L.ui[r], L.ir[r], L.ii[r]);
  }
}

// Fixed-point solve for the quad's env; every lane of the quad leaves with the
// same iteration count and its own converged currents in L.ir / L.ii.
template <int J>
__device__ __forceinline__ int pf_solve(const PFShared<J>& S, const pgw_pf_params& p, int q,
                                        PFLane<J>& L, bool pred, double pc) {
  constexpr int R = QuadDims<J>::R;
  if (pred) {
    // quadratic Lagrange interpolation of the 3 reference solutions at pc
    const double x0 = p.pred_p[0], x1 = p.pred_p[1], x2 = p.pred_p[2];
    const double w0 = ((pc - x1) * (pc - x2)) / ((x0 - x1) * (x0 - x2));
    const double w1 = ((pc - x0) * (pc - x2)) / ((x1 - x0) * (x1 - x2));
    const double w2 = ((pc - x0) * (pc - x1)) / ((x2 - x0) * (x2 - x1));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int k = 4 * r + q;
      L.ur[r] = w0 * S.Upred[0][k].x + w1 * S.Upred[1][k].x + w2 * S.Upred[2][k].x;
      L.ui[r] = w0 * S.Upred[0][k].y + w1 * S.Upred[1][k].y + w2 * S.Upred[2][k].y;
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      L.ur[r] = S.U0[4 * r + q].x;
      L.ui[r] = S.U0[4 * r + q].y;
    }
  }
  const double tol2 = p.tol * p.tol;
  int it = 0;
  while (it < p.max_iter) {
    ++it;
    // compiler-only fence: keeps the loop-invariant LDS tables from being
    // hoisted into (and spilled out of) registers
    asm volatile("" ::: "memory");
    pf_own_currents<J>(S, q, L);
    double Ir[J], Ii[J];
    quad_gather<J>(L, Ir, Ii);
    double err2 = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int k = 4 * r + q;
      double ar = S.U0[k].x, ai = S.U0[k].y;
      const double2* w = S.W + k * J;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const double2 wk = w[j];
        ar = fma(wk.x, Ir[j], ar);
        ar = fma(-wk.y, Ii[j], ar);
        ai = fma(wk.x, Ii[j], ai);
        ai = fma(wk.y, Ir[j], ai);
      }
      const double dr = ar - L.ur[r], di = ai - L.ui[r];
      const double e2 = (dr * dr + di * di) * S.thr[k].w;
      err2 = (e2 > err2) ? e2 : err2;
      L.ur[r] = ar;
      L.ui[r] = ai;
    }
    err2 = quad_max(err2);
    if (err2 < tol2) break;
  }
  pf_own_currents<J>(S, q, L);
  return it;
}

// |V| pu of output row o: V0 + sum_k G[o][k] I_k, each lane summing its own
// elements, then a quad sum (all four lanes return the value).
template <int J>
__device__ __forceinline__ double pf_node_pu(const PFShared<J>& S, const pgw_pf_tables& t, int o,
                                             int q, const PFLane<J>& L) {
  double vr = 0.0, vi = 0.0;
  const bool lds = o < kMaxOutLds;
#pragma unroll
  for (int r = 0; r < QuadDims<J>::R; ++r) {
    const int k = 4 * r + q;
    if (k < J) {
      double gx, gy;
      if (lds) {
        gx = S.G[o * J + k].x;
        gy = S.G[o * J + k].y;
      } else {
        gx = t.G[2 * (o * J + k)];
        gy = t.G[2 * (o * J + k) + 1];
      }
      vr = fma(gx, L.ir[r], vr);
      vr = fma(-gy, L.ii[r], vr);
      vi = fma(gx, L.ii[r], vi);
      vi = fma(gy, L.ir[r], vi);
    }
  }
  vr = quad_sum(vr);
  vi = quad_sum(vi);
  const double v0r = lds ? S.V0[o].x : t.V0[2 * o], v0i = lds ? S.V0[o].y : t.V0[2 * o + 1];
  vr = v0r + vr;
  vi = v0i + vi;
  return sqrt(vr * vr + vi * vi) * (lds ? S.inv_vbase_out[o] : t.inv_vbase_out[o]);
}

template <int J>
__device__ __forceinline__ void pf_store_u(const pgw_pf_tables& t, int64_t e, int q,
                                           const PFLane<J>& L) {
#pragma unroll
  for (int r = 0; r < QuadDims<J>::R; ++r) {
    const int k = 4 * r + q;
    if (k < J) {
      t.U_out[2 * (e * J + k)] = L.ur[r];
      t.U_out[2 * (e * J + k) + 1] = L.ui[r];
    }
  }
}

// Own element powers (opendss.py:107-129; OpenDSS WNominal = kW*1000/nphases).
template <int J>
__device__ __forceinline__ void pf_element_powers(const pgw_pf_params& p, const double* cp,
                                                  const double* cq, int q, PFLane<J>& L) {
#pragma unroll
  for (int r = 0; r < QuadDims<J>::R; ++r) {
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

constexpr int kEnvsPerBlock = kBlock / 4;

template <int J>
__global__ void __launch_bounds__(kBlock) k_pf_solve(pgw_pf_params p, pgw_pf_tables t, int64_t n,
                                                     const double* __restrict__ ctrl_p,
                                                     const double* __restrict__ ctrl_q,
                                                     double* __restrict__ v_out,
                                                     int32_t* __restrict__ iters) {
  __shared__ PFShared<J> S;
  const int n_lds = p.n_out < kMaxOutLds ? p.n_out : kMaxOutLds;
  pf_stage<J>(S, p, t, n_lds);
  __syncthreads();
  const int q = threadIdx.x & 3;
  const int64_t e = (int64_t)blockIdx.x * kEnvsPerBlock + (threadIdx.x >> 2);
  if (e >= n) return;                      // whole quads exit together
  double cp[PGW_PF_MAX_CTRL], cq[PGW_PF_MAX_CTRL];
#pragma unroll
  for (int c = 0; c < PGW_PF_MAX_CTRL; ++c) {
    cp[c] = (c < p.n_ctrl && ctrl_p) ? ctrl_p[(int64_t)c * n + e] : 0.0;
    cq[c] = (c < p.n_ctrl && ctrl_q) ? ctrl_q[(int64_t)c * n + e] : 0.0;
  }
  PFLane<J> L;
  pf_element_powers<J>(p, cp, cq, q, L);
  const int it = pf_solve<J>(S, p, q, L, t.U_pred != nullptr && p.n_ctrl == 1, cp[0]);
  for (int o = 0; o < p.n_out; ++o) {
    const double v = pf_node_pu<J>(S, t, o, q, L);
    if (q == 0) v_out[(int64_t)o * n + e] = v;
  }
  if (t.U_out) pf_store_u<J>(t, e, q, L);
  if (iters && q == 0) iters[e] = it;
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

// K2: one quad per env -- bus loads (multiagent_env.py:171-181), power flow
// (opendss.py:80-135), CoordinatedMultiBuildingControlEnv.reward_transform
// (train.py:51-63, 71-88) applied to the agent rewards in place.
template <int J>
__global__ void __launch_bounds__(kBlock) k_coord_pf(pgw_coord_params p, pgw_pf_params pf,
                                                     pgw_pf_tables pft, int64_t n,
                                                     pgw_coord_buffers b) {
  __shared__ PFShared<J> S;
  const int n_lds = pf.n_out < kMaxOutLds ? pf.n_out : kMaxOutLds;
  pf_stage<J>(S, pf, pft, n_lds);
  __syncthreads();
  const int q = threadIdx.x & 3;
  const int64_t e = (int64_t)blockIdx.x * kEnvsPerBlock + (threadIdx.x >> 2);
  if (e >= n) return;
  double cp[PGW_PF_MAX_CTRL], cq[PGW_PF_MAX_CTRL];
#pragma unroll
  for (int c = 0; c < PGW_PF_MAX_CTRL; ++c) {
    cp[c] = 0.0;
    cq[c] = 0.0;
  }
  for (int a = 0; a < p.n_agents; ++a) {
    const double rp = b.agent_power[(int64_t)a * n + e];
    const int slot = p.agent_ctrl[a];
#pragma unroll
    for (int c = 0; c < PGW_PF_MAX_CTRL; ++c) cp[c] = (c == slot) ? cp[c] + rp : cp[c];
  }
  PFLane<J> L;
  pf_element_powers<J>(pf, cp, cq, q, L);
  const int it = pf_solve<J>(S, pf, q, L, pft.U_pred != nullptr && pf.n_ctrl == 1, cp[0]);
  double vsel = 0.0;
  for (int o = 0; o < pf.n_out; ++o) {
    const double v = pf_node_pu<J>(S, pft, o, q, L);
    if (b.v_out && q == 0) b.v_out[(int64_t)o * n + e] = v;
    vsel = (o == p.vv_row) ? v : vsel;
  }
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

template <template <int> class K, typename... Args>
int32_t launch_m(int m, dim3 grid, hipStream_t stream, Args... args) {
  dim3 blk(kBlock);
  if (m <= 4) hipLaunchKernelGGL(K<4>::fn, grid, blk, 0, stream, args...);
  else if (m <= 8) hipLaunchKernelGGL(K<8>::fn, grid, blk, 0, stream, args...);
  else if (m <= 12) hipLaunchKernelGGL(K<12>::fn, grid, blk, 0, stream, args...);
  else if (m <= 14) hipLaunchKernelGGL(K<14>::fn, grid, blk, 0, stream, args...);
  else hipLaunchKernelGGL(K<16>::fn, grid, blk, 0, stream, args...);
  return check_launch("pgw power-flow kernel");
}

template <int M>
struct PFKernel {
  static constexpr auto fn = k_pf_solve<M>;
};
template <int M>
struct CoordPFKernel {
  static constexpr auto fn = k_coord_pf<M>;
};

// padded element count actually used by the device tables for a given m
static int padded_m(int m) { return m <= 4 ? 4 : m <= 8 ? 8 : m <= 12 ? 12 : m <= 14 ? 14 : 16; }

}  // namespace pgw

using namespace pgw;

extern "C" {

int32_t pgw_pf_padded_m(int32_t m) { return padded_m(m); }

int32_t pgw_pf_solve(const pgw_pf_params* p, const pgw_pf_tables* t, int64_t n,
                     const double* ctrl_p, const double* ctrl_q, double* v_out, int32_t* iters,
                     void* stream) {
  PGW_REQUIRE(p && t && t->W && t->U0 && v_out && n >= 0, "pgw_pf_solve: null argument");
  PGW_REQUIRE(p->m >= 1 && p->m <= PGW_PF_MAX_M && p->m == padded_m(p->m),
              "pgw_pf_solve: m=%d must be one of 4,8,12,14,16 (pad the tables)", p->m);
  PGW_REQUIRE(p->n_ctrl >= 0 && p->n_ctrl <= PGW_PF_MAX_CTRL, "pgw_pf_solve: bad n_ctrl");
  PGW_REQUIRE(p->n_out == 0 || (t->G && t->V0 && t->inv_vbase_out), "pgw_pf_solve: missing G/V0");
  PGW_REQUIRE(p->max_iter >= 1, "pgw_pf_solve: max_iter < 1");
  if (n == 0) return PGW_OK;
  return launch_m<PFKernel>(p->m, dim3(grid_for(4 * n)), (hipStream_t)stream, *p, *t, n, ctrl_p,
                            ctrl_q, v_out, iters);
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
  return launch_m<CoordPFKernel>(pf->m, dim3(grid_for(4 * n)), st, *p, *pf, *pft, n, b);
}

}  // extern "C"
