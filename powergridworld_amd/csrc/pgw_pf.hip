// Batched distribution power flow + the fused coordinated multi-building step.
//
// Power flow (replaces the OpenDSS snap solve behind opendss.py:80-165): per env,
// fixed-point current injection on the m load-element voltages
//     U <- U0 + W f(U),   f = OpenDSS PQ-load current law (model 1),
// with W = -C Z C^T, U0 = C V0 precomputed on the host (pgw_feeder.cpp) and
// shared by every env.  W is wave-uniform, so its loads are scalar loads; the
// per-env state (U, I) lives in registers: one thread per env, M (the element
// count rounded up to an instantiated size) fully unrolled.
#include "pgw_common.h"

namespace pgw {

template <int M>
struct PFState {
  double ur[M], ui[M];   // element voltages (V)
};

// OpenDSS Load.DoConstantPQLoad for every element: I_k = f_k(U_k).
template <int M>
__device__ __forceinline__ void pf_currents(const pgw_pf_params& p, const double sw[M],
                                            const double sv[M], const PFState<M>& s,
                                            double ir[M], double ii[M]) {
#pragma unroll
  for (int k = 0; k < M; ++k) {
    const double vb = p.vbase[k];
    const double ur = s.ur[k], ui = s.ui[k];
    const double mag2 = ur * ur + ui * ui;
    const double lo = p.vlow[k] * vb, mn = p.vmin[k] * vb, mx = p.vmax[k] * vb;
    if (mag2 > mn * mn && mag2 <= mx * mx) {
      // constant PQ: I = conj(S) / conj(U) = conj(S) U / |U|^2
      const double inv = 1.0 / mag2;
      ir[k] = (sw[k] * ur + sv[k] * ui) * inv;
      ii[k] = (sw[k] * ui - sv[k] * ur) * inv;
    } else {
      // constant Z:  Yeq = conj(S)/Vbase^2, scaled by 1/Vminpu^2 or 1/Vmaxpu^2
      const double vb2 = vb * vb;
      double yr = sw[k] / vb2, yi = -sv[k] / vb2;
      if (mag2 > lo * lo) {
        const double v = (mag2 <= mn * mn) ? p.vmin[k] : p.vmax[k];
        const double v2 = v * v;
        yr = yr / v2;
        yi = yi / v2;
      }
      ir[k] = yr * ur - yi * ui;
      ii[k] = yr * ui + yi * ur;
    }
  }
}

// Solve one env.  sw/sv: per-element W / var.  Returns the iteration count and
// leaves the converged element currents in ir/ii.
template <int M>
__device__ __forceinline__ int pf_solve(const pgw_pf_params& p, const pgw_pf_tables& t,
                                        const double sw[M], const double sv[M], double ir[M],
                                        double ii[M]) {
  PFState<M> s;
#pragma unroll
  for (int k = 0; k < M; ++k) {
    s.ur[k] = t.U0[2 * k];
    s.ui[k] = t.U0[2 * k + 1];
  }
  const double tol2 = p.tol * p.tol;
  int it = 0;
  while (it < p.max_iter) {
    ++it;
    pf_currents<M>(p, sw, sv, s, ir, ii);
    double err2 = 0.0;
#pragma unroll
    for (int k = 0; k < M; ++k) {
      double ar = t.U0[2 * k], ai = t.U0[2 * k + 1];
      const double* w = t.W + 2 * M * k;
#pragma unroll
      for (int j = 0; j < M; ++j) {
        const double wr = w[2 * j], wi = w[2 * j + 1];
        ar = fma(wr, ir[j], ar);
        ar = fma(-wi, ii[j], ar);
        ai = fma(wr, ii[j], ai);
        ai = fma(wi, ir[j], ai);
      }
      const double dr = ar - s.ur[k], di = ai - s.ui[k];
      const double vb = p.vbase[k];
      const double e2 = (dr * dr + di * di) / (vb * vb);
      err2 = (e2 > err2) ? e2 : err2;
      s.ur[k] = ar;
      s.ui[k] = ai;
    }
    if (err2 < tol2) break;
  }
  pf_currents<M>(p, sw, sv, s, ir, ii);
  return it;
}

// |V| pu at output row r: V = V0[r] + G[r] . I
template <int M>
__device__ __forceinline__ double pf_node_pu(const pgw_pf_tables& t, int r, const double ir[M],
                                             const double ii[M]) {
  double vr = t.V0[2 * r], vi = t.V0[2 * r + 1];
  const double* g = t.G + 2 * M * r;
#pragma unroll
  for (int j = 0; j < M; ++j) {
    vr = fma(g[2 * j], ir[j], vr);
    vr = fma(-g[2 * j + 1], ii[j], vr);
    vi = fma(g[2 * j], ii[j], vi);
    vi = fma(g[2 * j + 1], ir[j], vi);
  }
  return sqrt(vr * vr + vi * vi) * t.inv_vbase_out[r];
}

template <int M>
__device__ __forceinline__ void pf_element_powers(const pgw_pf_params& p, const double* cp,
                                                  const double* cq, double sw[M], double sv[M]) {
#pragma unroll
  for (int k = 0; k < M; ++k) {
    double kw = p.base_kw[k], kvar = p.base_kvar[k];
    const int c = p.elem_ctrl[k];
    if (c >= 0) {
      kw = kw + cp[c];
      kvar = kvar + cq[c];
    }
    sw[k] = (kw * 1000.0) / p.nph[k];
    sv[k] = (kvar * 1000.0) / p.nph[k];
  }
}

template <int M>
__global__ void __launch_bounds__(kBlock) k_pf_solve(pgw_pf_params p, pgw_pf_tables t, int64_t n,
                                                     const double* __restrict__ ctrl_p,
                                                     const double* __restrict__ ctrl_q,
                                                     double* __restrict__ v_out,
                                                     int32_t* __restrict__ iters) {
  int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  double cp[PGW_PF_MAX_CTRL], cq[PGW_PF_MAX_CTRL];
#pragma unroll
  for (int c = 0; c < PGW_PF_MAX_CTRL; ++c) {
    cp[c] = (c < p.n_ctrl && ctrl_p) ? ctrl_p[(int64_t)c * n + e] : 0.0;
    cq[c] = (c < p.n_ctrl && ctrl_q) ? ctrl_q[(int64_t)c * n + e] : 0.0;
  }
  double sw[M], sv[M], ir[M], ii[M];
  pf_element_powers<M>(p, cp, cq, sw, sv);
  int it = pf_solve<M>(p, t, sw, sv, ir, ii);
  for (int r = 0; r < p.n_out; ++r) v_out[(int64_t)r * n + e] = pf_node_pu<M>(t, r, ir, ii);
  if (iters) iters[e] = it;
}

// ============================================================ fused coordinated step
// MultiAgentEnv.step (multiagent_env.py:151-212) for n_agents identical
// MultiComponentEnv agents (base.py:114-156) of {building, pv, storage}
// (scenarios/buildings.py:11-72), the power flow on the agents' common bus and
// CoordinatedMultiBuildingControlEnv.reward_transform (examples/marl/openai/
// train.py:51-88).  One thread per env; all agent state stays in registers.
template <int M>
__global__ void __launch_bounds__(kBlock) k_coord_step(pgw_coord_params p, pgw_pf_params pf,
                                                       pgw_pf_tables pft, pgw_coord_step_info s,
                                                       int64_t n, pgw_coord_buffers b) {
  int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  double cp[PGW_PF_MAX_CTRL], cq[PGW_PF_MAX_CTRL];
#pragma unroll
  for (int c = 0; c < PGW_PF_MAX_CTRL; ++c) {
    cp[c] = 0.0;
    cq[c] = 0.0;
  }
  double rew[PGW_MAX_AGENTS];
  const double pv_ob = pv_obs(p.pv, s.pv_pmax);
  const BuildingExt xv = {1.0, 1.0, 1.0, __builtin_huge_val()};

#pragma unroll 1
  for (int a = 0; a < p.n_agents; ++a) {
    pgw_mat act = b.action;
    act.ptr += a * b.act_stride_agent;
    pgw_mat obs = b.obs;
    obs.ptr += a * b.obs_stride_agent;
    double agent_rp = 0.0, agent_rew = 0.0;
    double r_bld = 0.0;
    for (int ci = 0; ci < p.n_comp; ++ci) {
      const int comp = p.comp_order[ci];
      if (comp == 0) {
        // ---- building (five_zone_rom_env.py:183-225), fresh reward (base.py:137)
        double av[6], xs[5], T[5];
#pragma unroll
        for (int j = 0; j < 6; ++j) {
          double v = ld(act, e, p.act_bld + j);
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
        building_write_obs(p.bld, T, s.ex_next, pc, xv,
                           [&](int j, double v) { st(obs, e, p.obs_bld + j, v); });
        agent_rp = agent_rp + pc;
      } else if (comp == 1) {
        // ---- PV (pv_profile_env.py:133-148)
        st(obs, e, p.obs_pv, pv_ob);
        agent_rp = agent_rp + pv_real_power(p.pv, ld(act, e, p.act_pv), s.pv_pmax);
      } else {
        // ---- storage (energy_storage_env.py:131-157)
        double soc = b.soc[(int64_t)a * n + e];
        const double power = battery_step(p.bat, ld(act, e, p.act_bat), soc);
        b.soc[(int64_t)a * n + e] = soc;
        st(obs, e, p.obs_bat, battery_obs(p.bat, soc));
        agent_rp = agent_rp + (-power);
      }
    }
    // MultiComponentEnv.step_reward: 0. + building + pv(0) + storage(0)
    for (int ci = 0; ci < p.n_comp; ++ci) agent_rew = agent_rew + (p.comp_order[ci] == 0 ? r_bld : 0.0);
    b.agent_power[(int64_t)a * n + e] = agent_rp;
    // load_p[bus] += agent.real_power (multiagent_env.py:171-181)
    const int slot = p.agent_ctrl[a];
#pragma unroll
    for (int c = 0; c < PGW_PF_MAX_CTRL; ++c)
      if (c == slot) cp[c] = cp[c] + agent_rp;
    rew[a < PGW_MAX_AGENTS ? a : 0] = agent_rew;
  }

  // ---- power flow on the bus loads (opendss.py:80-135)
  double sw[M], sv[M], ir[M], ii[M];
  pf_element_powers<M>(pf, cp, cq, sw, sv);
  const int it = pf_solve<M>(pf, pft, sw, sv, ir, ii);
  double vsel = 0.0;
  for (int r = 0; r < pf.n_out; ++r) {
    const double v = pf_node_pu<M>(pft, r, ir, ii);
    if (b.v_out) b.v_out[(int64_t)r * n + e] = v;
    if (r == p.vv_row) vsel = v;
  }
  if (b.iters) b.iters[e] = it;

  // ---- CoordinatedMultiBuildingControlEnv.reward_transform (train.py:51-63,71-88)
  double vv = 0.0;
  if (p.coordinated) {
    vv = pymax(pymax(0.0, p.vv_lo - vsel), vsel - p.vv_hi);
    if (b.vv) b.vv[e] = vv;
  }
  const double share = (vv * p.vv_penalty) / (double)p.n_agents;
#pragma unroll 1
  for (int a = 0; a < p.n_agents; ++a) {
    double r = rew[a];
    if (p.coordinated) r = r - share;
    b.reward[(int64_t)a * n + e] = r;
  }
}

template <template <int> class K, typename... Args>
int32_t launch_m(int m, int64_t n, hipStream_t stream, Args... args) {
  dim3 g(grid_for(n)), blk(kBlock);
  if (n <= 0) return PGW_OK;
  if (m <= 4) hipLaunchKernelGGL(K<4>::fn, g, blk, 0, stream, args...);
  else if (m <= 8) hipLaunchKernelGGL(K<8>::fn, g, blk, 0, stream, args...);
  else if (m <= 12) hipLaunchKernelGGL(K<12>::fn, g, blk, 0, stream, args...);
  else if (m <= 14) hipLaunchKernelGGL(K<14>::fn, g, blk, 0, stream, args...);
  else hipLaunchKernelGGL(K<16>::fn, g, blk, 0, stream, args...);
  return check_launch("pgw power-flow kernel");
}

template <int M>
struct PFKernel {
  static constexpr auto fn = k_pf_solve<M>;
};
template <int M>
struct CoordKernel {
  static constexpr auto fn = k_coord_step<M>;
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
  return launch_m<PFKernel>(p->m, n, (hipStream_t)stream, *p, *t, n, ctrl_p, ctrl_q, v_out, iters);
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
  for (int a = 0; a < p->n_agents; ++a)
    PGW_REQUIRE(p->agent_ctrl[a] < pf->n_ctrl, "pgw_coord_step: agent_ctrl out of range");
  for (int c = 0; c < p->n_comp; ++c) {
    int k = p->comp_order[c];
    PGW_REQUIRE(k >= 0 && k <= 2, "pgw_coord_step: bad comp_order");
    if (k == 0) PGW_REQUIRE(b.x && p->act_bld >= 0 && p->bld.n_obs <= PGW_BLD_MAX_OBS, "pgw_coord_step: building");
    if (k == 2) PGW_REQUIRE(b.soc && p->act_bat >= 0, "pgw_coord_step: storage");
  }
  return launch_m<CoordKernel>(pf->m, n, (hipStream_t)stream, *p, *pf, *pft, *s, n, b);
}

}  // extern "C"
