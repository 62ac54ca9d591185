// Batched distribution power flow + the coordinated multi-building step.
//
// Power flow (replaces the OpenDSS snap solve behind opendss.py:80-165): per env,
// fixed-point current injection on the m load-element voltages
//     U <- U0 + W f(U),   f = OpenDSS PQ-load current law (model 1),
// with W = -C Z C^T, U0 = C V0 precomputed on the host (pgw_feeder.cpp) and
// shared by every env.  The kernels iterate in per unit of each element's base
// voltage (u = U / vb, W'_ik = W_ik / vb_i, s_k = conj(S_k) / vb_k): the band
// limits and the convergence test then need no per-element scale.
//
// Layout: ONE LANE PER ENV, everything in registers.  The lane keeps its m
// element voltages; the operands shared by all envs -- W' (as the three real
// matrices of the 3-multiply complex product: Re = Wr Ir - Wi Ii, Im = (Wr+Wi)
// (Ir+Ii) - Wr Ir - Wi Ii), u0 and the element powers -- stay RESIDENT in VGPRs
// for the whole solve, 16 entries per register pair (entry e in lane e % 16 of
// each 16-lane row of pair e / 16), and reach the FMA through a DPP broadcast
// operand: v_fmac_f64_dpp acc, w, x row_newbcast:(e % 16).  So one iteration is
// ~1000 fp64 VALU instructions per 64 envs with no memory or scalar traffic
// (588 FMAs of the matvec).  Lanes whose env has converged leave the loop (exec
// mask), so each env's result and iteration count are those of iterating it
// alone.  On MI355X fp64 MFMA has the same peak as the fp64 VALU and does not
// co-issue with it (measured, profiles/r01/), so the matrix cores gain nothing.
//
// Coordinated step (the BASELINE C4 path) = two launches on one stream:
//   k_coord_agents  one thread per (env, agent): building + PV + storage step,
//                   obs/state writes, agent real power and (pre-transform) reward
//                   -- pure HBM streaming, 5x the waves of a per-env kernel;
//   k_coord_pf      one lane per env: bus loads = sum of agent powers, power
//                   flow, voltage-violation penalty folded into the rewards.
#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <type_traits>
#include <atomic>
#include <vector>

#include "pgw_common.h"

// pgw_debug_pf_trace set: k_coord_pf_od launches its trace instantiation
static std::atomic<bool> g_pf_trace_on{false};

namespace pgw {

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// ---- resident operand block ------------------------------------------------
// Packed block (pgw_pf_pack, doubles), M = padded element count, T = M(M+1)/2:
//   [0, 3T)      part c of the upper triangle of W'' = W_ik / (vb_i vb_k), which is
//                complex symmetric: c = 0 Re, 1 Im, 2 Re + Im; entry (i <= k) at
//                c T + i M - i(i-1)/2 + (k - i)
//   [3T, +3M)    u0re[i], u0im[i], u0re[i] + u0im[i]   (u0 = U0 / vb)
//   [.., +3M)    vlow^2, vmin^2, vmax^2 per element (pu^2)
//   [.., +2M+2)  output row 0 of the tables (pu): G re, im; V0 re, im
// The iteration runs on u = U / vb and the scaled currents I' = I vb =
// conj(S) u g, so u_i = u0_i + sum_k W''_ik I'_k.
template <int M> struct PFBlock {
  static constexpr int kTri = M * (M + 1) / 2;
  static constexpr int kU0re = 3 * kTri, kU0im = kU0re + M, kU0sum = kU0im + M;
  static constexpr int kLo2 = kU0sum + M, kMn2 = kLo2 + M, kMx2 = kMn2 + M;
  static constexpr int kG0re = kMx2 + M, kG0im = kG0re + M, kV0re = kG0im + M, kV0im = kV0re + 1;
  static constexpr int kSize = kV0im + 1;
  static constexpr int kPairs = (kSize + 15) / 16;
};
static int64_t pf_block_size(int m) { return 3LL * m * (m + 1) / 2 + 8LL * m + 2; }

// Per-launch scalars derived on the host from pgw_pf_params (pu).
struct PFArgs {
  double sr0[PGW_PF_MAX_M], si0[PGW_PF_MAX_M];   // s0 = conj(S_base) per phase (W, var)
  double fr[PGW_PF_MAX_M], fi[PGW_PF_MAX_M];     // d s / d (ctrl kW, kvar): slot-0 elements
  double kw[PGW_PF_MAX_M], kvar[PGW_PF_MAX_M], nph[PGW_PF_MAX_M];
  int32_t ctrl[PGW_PF_MAX_M];
  double lo2, mn2, mx2;                          // band limits when uniform (pu^2)
  double tol2;
  double pred_x0, pred_inv_h;
  int32_t pred_n, use_pred, max_iter, n_ctrl, n_out;
};
constexpr int kSPairs = (4 * PGW_PF_MAX_M + 15) / 16;   // resident s0 / f entries

// The DPP-broadcast groups (generated: gen_pf_dpp.py).  Entry e of a resident
// table lives in lane e % 16 of every 16-lane row of register pair e / 16 and is
// fed to its instruction with row_newbcast:(e % 16).
// Output-row operands in resident form (pf_rows_out): slot j of a row (V0 re,
// V0 im, G re of every element, G im of every element) in lane j % 16 of pair
// j / 16.
template <int M> struct PFRow {
  static constexpr int kPairs = (2 * M + 2 + 15) / 16;
};
#include "pgw_pf_dpp.inc"

__device__ __forceinline__ double fast_rcp(double m) {
  // v_rcp_f64 + two Newton steps (~1 ulp; the exact IEEE divide sequence costs
  // ~3x more and the PF is iterated to a tolerance anyway)
  double r = __builtin_amdgcn_rcp(m);
  double e = fma(-m, r, 1.0);
  r = fma(r, e, r);
  e = fma(-m, r, 1.0);
  return fma(r, e, r);
}

// Per-lane solver state.  UB: every element has the same (vlow, vmin, vmax);
// GC: more than one controllable slot (per-lane s for every element).
template <int M, bool UB, bool GC> struct PFSolver {
  using Lo = PFBlock<M>;
  static constexpr int NR = Lo::kPairs;
  double w[NR];            // resident block
  double sres[kSPairs];    // resident s0r, s0i, fr, fi (entry k, M+k, 2M+k, 3M+k)
  double ur[M], ui[M];     // element voltages (pu)
  double sr[GC ? M : 1], si[GC ? M : 1];
  double pc, qc;           // slot-0 controllable kW / kvar of the env
  double lo2, mn2, mx2, tol2;

  __device__ __forceinline__ void load(const PFArgs& a, const double* block) {
    const int l = threadIdx.x & 15;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int e = 16 * j + l;
      w[j] = e < Lo::kSize ? block[e] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < kSPairs; ++j) {
      const int e = 16 * j + l;              // 4 tables of M entries
      const int t = e / M, k = e - t * M;
      const double* src = t == 0 ? a.sr0 : t == 1 ? a.si0 : t == 2 ? a.fr : a.fi;
      sres[j] = t < 4 ? src[k] : 0.0;
    }
    lo2 = a.lo2;
    mn2 = a.mn2;
    mx2 = a.mx2;
    tol2 = a.tol2;
  }

  // element powers of the env (opendss.py:107-129; OpenDSS WNominal = kW*1000/nphases)
  __device__ __forceinline__ void powers(const PFArgs& a, const double* cp, const double* cq,
                                         double scale) {
    pc = cp[0];
    qc = cq[0];
    if constexpr (GC) {
#pragma unroll
      for (int k = 0; k < M; ++k) {
        const int c = a.ctrl[k];
        double p = 0.0, q = 0.0;
#pragma unroll
        for (int s = 0; s < PGW_PF_MAX_CTRL; ++s) {
          p = (c == s) ? cp[s] : p;
          q = (c == s) ? cq[s] : q;
        }
        sr[k] = ((a.kw[k] * scale + p) * 1000.0) / a.nph[k];
        si[k] = -(((a.kvar[k] * scale + q) * 1000.0) / a.nph[k]);
      }
    }
  }

  // OpenDSS Load.DoConstantPQLoad (model 1), in pu: I' = I vb = conj(S) u g with
  //   g = 1/|u|^2 for vmin < |u| <= vmax, the constant-Z scales 1/vmin^2 below
  //   vmin and 1/vmax^2 above vmax -- i.e. 1/clamp(|u|^2, vmin^2, vmax^2), exact
  //   at both band edges -- and 1 at or below vlow.
  template <int K>
  __device__ __forceinline__ void current(double& ir, double& ii) const {
    double s_r, s_i;
    if constexpr (GC) {
      s_r = sr[K];
      s_i = si[K];
    } else {
      pf_power<M, K>(s_r, s_i, sres, pc, qc);
    }
    double vlo2, vmn2, vmx2;
    band<K>(vlo2, vmn2, vmx2);
    const double m2 = fma(ui[K], ui[K], ur[K] * ur[K]);
    double mc = fmin(fmax(m2, vmn2), vmx2);
    mc = (m2 <= vlo2) ? 1.0 : mc;
    const double g = fast_rcp(mc);
    const double gr = g * ur[K], gi = g * ui[K];
    ir = fma(s_r, gr, -(s_i * gi));
    ii = fma(s_r, gi, s_i * gr);
  }

  // Initial guess: quadratic through the 3 predictor grid points nearest pc, or u0.
  // Band limits of element K (pu^2).
  template <int K>
  __device__ __forceinline__ void band(double& vlo2, double& vmn2, double& vmx2) const {
    if constexpr (UB) {
      vlo2 = lo2;
      vmn2 = mn2;
      vmx2 = mx2;
    } else {
      pf_band<M, K>(vlo2, vmn2, vmx2, w);
    }
  }

  // Band of every element in 2 bits (0 |u| <= vlow, 1 <= vmin, 2 <= vmax, 3 above),
  // the states the load law switches between.  Whole wave (DPP in pf_band).
  __device__ __forceinline__ int32_t signature() const {
    uint32_t sg = 0;
    static_for<0, M>([&](auto k) {
      double vlo2, vmn2, vmx2;
      band<k>(vlo2, vmn2, vmx2);
      const double m2 = fma(ui[k], ui[k], ur[k] * ur[k]);
      const uint32_t b = (uint32_t)(m2 > vlo2) + (uint32_t)(m2 > vmn2) + (uint32_t)(m2 > vmx2);
      sg |= b << (2 * k);
    });
    return (int32_t)sg;
  }

  // Predictor record c (pgw_pf_pred_pack): u_c (fp64) and d1, d2 (fp32).
  struct Rec {
    double2 u[M];
    float2 d1[M], d2[M];
  };
  __device__ __forceinline__ static void pred_load(const double* rec, int c, Rec& R) {
    const char* r = reinterpret_cast<const char*>(rec) + (int64_t)c * (32 * M);
    const double2* v = reinterpret_cast<const double2*>(r);
    const float2* d1 = reinterpret_cast<const float2*>(r + 16 * M);
    const float2* d2 = reinterpret_cast<const float2*>(r + 24 * M);
#pragma unroll
    for (int k = 0; k < M; ++k) {
      R.u[k] = v[k];
      R.d1[k] = d1[k];
      R.d2[k] = d2[k];
    }
  }
  // Its quadratic at grid coordinate g: u = u_c + t (d1/2 + t d2/2), t = g - c.
  __device__ __forceinline__ void pred_eval(const Rec& R, int c, double g) {
    const double t = g - (double)c;
    const double h1 = 0.5 * t, h2 = 0.5 * t * t;
#pragma unroll
    for (int k = 0; k < M; ++k) {
      ur[k] = fma(h2, (double)R.d2[k].x, fma(h1, (double)R.d1[k].x, R.u[k].x));
      ui[k] = fma(h2, (double)R.d2[k].y, fma(h1, (double)R.d1[k].y, R.u[k].y));
    }
  }
  __device__ __forceinline__ void pred_quad(const double* rec, int c, double g) {
    Rec R;
    pred_load(rec, c, R);
    pred_eval(R, c, g);
  }

  // Initial guess: per-env U_init; or the predictor -- the quadratic through 3
  // grid solutions, the stencil chosen per grid segment by pgw_pf_pred_meta so
  // that it never straddles a load-band switch; or u0.
  // SPEC: load the nearest record speculatively with the segment metadata (the
  // fast kernel; the others keep the dependent loads, which need fewer VGPRs).
  template <bool SPEC = false>
  __device__ __forceinline__ void initial(const PFArgs& a, const pgw_pf_tables& t, int64_t e,
                                          bool valid) {
    if (t.U_init) {
      const double2* P = reinterpret_cast<const double2*>(t.U_init) + (valid ? e : 0) * M;
#pragma unroll
      for (int k = 0; k < M; ++k) {
        const double2 v = P[k];
        ur[k] = v.x;
        ui[k] = v.y;
      }
    } else if (a.use_pred) {
      const double g = (pc - a.pred_x0) * a.pred_inv_h;
      // the nearest record: what the segment's stencil choice is everywhere
      // but next to a load-band switch
      const int c0 = (int)fmin(fmax(rint(g), 1.0), (double)(a.pred_n - 2));
      if (SPEC && t.U_pred_meta) {
        // its loads go out together with the segment's metadata load (one L2
        // round trip instead of two); a lane whose segment picks another
        // centre reloads
        const int j = (int)fmin(fmax(floor(g), 0.0), (double)(a.pred_n - 2));
        const pgw_pred_meta m = t.U_pred_meta[j];
        Rec R;
        pred_load(t.U_pred, c0, R);
        const int c = (g - (double)j < m.tstar) ? m.left : m.right;
        if (c != c0) pred_load(t.U_pred, c, R);
        pred_eval(R, c, g);
      } else if (t.U_pred_meta) {
        const int j = (int)fmin(fmax(floor(g), 0.0), (double)(a.pred_n - 2));
        const pgw_pred_meta m = t.U_pred_meta[j];
        pred_quad(t.U_pred, (g - (double)j < m.tstar) ? m.left : m.right, g);
      } else {
        pred_quad(t.U_pred, c0, g);
      }
    } else {
      pf_u0<M>(ur, ui, w);
    }
  }

  // OpenDSS's compensation current (Load.CalcInjCurrentArray: the load's model-1
  // current less its Yeq stamped in Y), in pu: I' = (conj(S) g - y0') u -- the
  // operations and order of k_pf_general's model-1 path.
  template <int K>
  __device__ __forceinline__ void current_od(double y0r, double y0i, double& ir, double& ii) const {
    double s_r, s_i;
    pf_power<M, K>(s_r, s_i, sres, pc, qc);
    double vlo2, vmn2, vmx2;
    band<K>(vlo2, vmn2, vmx2);
    const double m2 = fma(ui[K], ui[K], ur[K] * ur[K]);
    double mc = fmin(fmax(m2, vmn2), vmx2);
    mc = (m2 <= vlo2) ? 1.0 : mc;
    const double g = fast_rcp(mc);
    const double cr = fma(s_r, g, -y0r), ci = fma(s_i, g, -y0i);
    ir = fma(cr, ur[K], -(ci * ui[K]));
    ii = fma(cr, ui[K], ci * ur[K]);
  }

  // Fixed-point iteration until max_k |du_k|^2 < tol^2 or max_iter.  The loop
  // is wave-uniform with the exec mask FULL: a lane disabled in EXEC is an
  // invalid DPP source, and every lane holds resident entries the others
  // broadcast from.  An env that has converged (or a lane past n) keeps its
  // voltages by select, so each env's result and iteration count are those of
  // iterating it alone.
  // The output voltages come from the currents of the LAST iteration (the
  // currents of the voltages it started from), as in OpenDSS, whose reported
  // node voltages are the solve V_{k+1} = Y^-1 I(V_k) that passed the
  // convergence test -- every node, output nodes included, from the same I.
  // KEEP = false (fast kernel, one output row): output node 0 is accumulated
  // inside the loop, column by column, in pf_node0's operation order.
  // KEEP = true (general kernels, any outputs): the currents are kept per lane.
  template <bool KEEP>
  __device__ __forceinline__ int iterate(int max_iter, bool valid, double& v0r, double& v0i,
                                         double (&lir)[M], double (&lii)[M]) {
    int it = 0, my_it = 0;
    bool done = !valid, conv_ok = !valid;
    v0r = v0i = 0.0;
    if constexpr (KEEP) {
#pragma unroll
      for (int k = 0; k < M; ++k) lir[k] = lii[k] = 0.0;
    }
    while (true) {
      double A[M], Bs[M], C[M], vr, vi;
      pf_acc_init<M>(A, C, w);
      if constexpr (!KEEP) pf_v0<M>(vr, vi, w);
#pragma unroll
      for (int i = 0; i < M; ++i) Bs[i] = 0.0;
      auto column = [&](auto k, double ir, double ii) {
        const double is = ir + ii;
        if constexpr (KEEP) {
          pf_column<M, decltype(k)::value>(A, Bs, C, w, ir, ii, is);
          lir[k] = done ? lir[k] : ir;
          lii[k] = done ? lii[k] : ii;
        } else {
          pf_column_v<M, decltype(k)::value>(A, Bs, C, vr, vi, w, ir, ii, is);
        }
      };
      // two elements at a time: their current-law chains (v_rcp_f64 + Newton)
      // are independent, so the scheduler interleaves them instead of stalling
      // on one dependent chain between two FMA blocks
      static_for<0, M / 2>([&](auto h) {
        constexpr int k0 = 2 * h, k1 = 2 * h + 1;
        double ir0, ii0, ir1, ii1;
        current<k0>(ir0, ii0);
        current<k1>(ir1, ii1);
        column(std::integral_constant<int, k0>{}, ir0, ii0);
        column(std::integral_constant<int, k1>{}, ir1, ii1);
      });
      if constexpr (M % 2) {
        double ir, ii;
        current<M - 1>(ir, ii);
        column(std::integral_constant<int, M - 1>{}, ir, ii);
      }
      bool conv = true;
#pragma unroll
      for (int i = 0; i < M; ++i) {
        const double nr = A[i] - Bs[i];
        const double ni = (C[i] - A[i]) - Bs[i];
        const double dr = nr - ur[i], di = ni - ui[i];
        conv &= fma(dr, dr, di * di) < tol2;
        ur[i] = done ? ur[i] : nr;
        ui[i] = done ? ui[i] : ni;
      }
      if constexpr (!KEEP) {
        v0r = done ? v0r : vr;
        v0i = done ? v0i : vi;
      }
      ++it;
      my_it = done ? my_it : it;
      conv_ok = conv_ok || (!done && conv);
      done = done || conv || it >= max_iter;
      if (__ballot(!done) == 0ull) break;
    }
    if constexpr (KEEP) pf_node0<M>(v0r, v0i, w, lir, lii);
    // an env stopped by max_iter before passing the test reports -iterations
    return conv_ok ? my_it : -my_it;
  }

};

// Debug phase trace (pgw_debug_pf_trace): when set, lane 0 of every k_coord_pf
// or k_pf_solve wave records wall_clock64() (100 MHz) at each phase boundary
// (the buffer holds 8 slots per wave of the launch).  Global, not flat, stores:
// a pending flat store counts against lgkmcnt too and would make the LDS waits
// after it conservative.
__device__ long long* g_pf_trace = nullptr;
__device__ __forceinline__ void pf_trace(long long* tr, int phase) {
  if (tr && (threadIdx.x & 63) == 0) {
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    typedef __attribute__((address_space(1))) long long* gptr;
    ((gptr)tr)[wave * 8 + phase] = wall_clock64();
  }
}

// |V| pu of output node o: V0 + sum_k G[o][k] I_k (wave-uniform G, V0 rows
// through the scalar cache).
typedef const __attribute__((address_space(4))) double* sdptr;
__device__ __forceinline__ sdptr scalar_ptr(const double* p) { return (sdptr)p; }

// (ir, ii: the scaled currents I' = I vb; the rows are pu-scaled on the host.
// The same operations in the same order as the resident node-0 group, so an
// output node gets bit-identical voltages whichever row it occupies.)
template <int M>
__device__ __forceinline__ double pf_node_pu(const pgw_pf_tables& t, int o, const double* ir,
                                             const double* ii) {
  const sdptr G = scalar_ptr(t.G) + 2 * M * o;
  double vr = scalar_ptr(t.V0)[2 * o], vi = scalar_ptr(t.V0)[2 * o + 1];
#pragma unroll
  for (int k = 0; k < M; ++k) {
    const double gr = G[2 * k], gi = G[2 * k + 1];
    vr = fma(gr, ir[k], vr);
    vr = fma(-gi, ii[k], vr);
    vi = fma(gr, ii[k], vi);
    vi = fma(gi, ir[k], vi);
  }
  return sqrt(fma(vi, vi, vr * vr));
}

// The general kernels' output rows, staged in LDS by the block in the resident
// row layout (PFRow: 16 kPairs doubles per row), copied before the solve so the
// loads overlap it.  A lane then loads slot (16 p + lane % 16) of each pair of
// a row: 2 x 512 B of LDS data per row and wave, where broadcast reads of the
// whole row (every lane all 2M + 2 operands) moved 15 KB and were bound by the
// LDS return bandwidth (0.26 us per row).
constexpr int kRowsLds = 4096;   // doubles (32 KB); more rows use pf_node_pu
template <int M>
__device__ __forceinline__ bool pf_rows_stage(const pgw_pf_tables& t, int n_out, double* s) {
  constexpr int S = 16 * PFRow<M>::kPairs;
  if (n_out * S > kRowsLds || n_out <= 1) return false;   // uniform
  // four entries per lane in flight per pass (branch-free sources), then
  // their LDS stores: one L2 round trip per 4 kBlock entries instead of one
  // per kBlock (the rolled loop waited for each load before the next)
  constexpr int kQ = 4;
  const int total = n_out * S;
  for (int base = 0; base < total; base += kQ * kBlock) {   // uniform
    double v[kQ];
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      const int i = base + q * kBlock + threadIdx.x;
      const int o = i / S, j = i - o * S;
      const bool has = i < total && j < 2 + 2 * M;
      const double* p = j < 2 ? t.V0 + (2 * o + j)
                              : t.G + (2 * M * o + (j < 2 + M ? 2 * (j - 2) : 2 * (j - 2 - M) + 1));
      v[q] = has ? *p : 0.0;
    }
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      const int i = base + q * kBlock + threadIdx.x;
      if (i < total) s[i] = v[q];
    }
  }
  return true;
}

// Output rows 1 .. n_out-1, f(o, |V_o|) called in row order.  From LDS: each
// row's operands are loaded into resident pairs (one 8-byte LDS read per pair)
// four rows ahead of use, and the rows are evaluated four at a time by DPP
// broadcast FMAs (pf_row4_dpp: eight independent chains; at 65 536 envs the
// kernel runs one wave per SIMD, which needs about eight DPP chains to
// approach the fp64 issue rate, tools/micro/fp64_issue.hip).  Per row the operations and their order are
// pf_node_pu's, so the values are bit-identical.
template <int M>
__device__ __forceinline__ void pf_row_load(const double* s, int o, double (&w)[PFRow<M>::kPairs]) {
  const double* r = s + 16 * PFRow<M>::kPairs * o + (threadIdx.x & 15);
#pragma unroll
  for (int p = 0; p < PFRow<M>::kPairs; ++p) w[p] = r[16 * p];
}
// SQ = false: f receives |V|^2 (fma(vi, vi, vr * vr), before pf_node_pu's
// sqrt) -- for extrema-only solves, whose min / max over the rows are the sqrt
// of the min / max of |V|^2 (sqrt is monotone and correctly rounded).
template <int M, bool SQ = true>
__device__ __forceinline__ double pf_mag(double vr, double vi) {
  const double m2 = fma(vi, vi, vr * vr);
  return SQ ? sqrt(m2) : m2;
}
template <int M, bool SQ = true, class F>
__device__ __forceinline__ void pf_rows_out(const pgw_pf_tables& t, bool rows_lds, const double* s,
                                            int n_out, const double (&ir)[M], const double (&ii)[M],
                                            F&& f) {
  if (!rows_lds) {   // (SQ only: the extrema-only caller needs the staged rows)
    if constexpr (SQ)
      for (int o = 1; o < n_out; ++o) f(o, pf_node_pu<M>(t, o, ir, ii));
    return;
  }
  constexpr int P = PFRow<M>::kPairs;
  double wa[P], wb[P], wc[P], wd[P], na[P], nb[P], nc[P], nd[P];
  const int last = n_out - 1;
  pf_row_load<M>(s, 1, wa);
  pf_row_load<M>(s, min(2, last), wb);
  pf_row_load<M>(s, min(3, last), wc);
  pf_row_load<M>(s, min(4, last), wd);
  int o = 1;
  for (; o + 4 <= n_out; o += 4) {
    pf_row_load<M>(s, min(o + 4, last), na);     // the next four rows in flight
    pf_row_load<M>(s, min(o + 5, last), nb);
    pf_row_load<M>(s, min(o + 6, last), nc);
    pf_row_load<M>(s, min(o + 7, last), nd);
    __builtin_amdgcn_sched_barrier(0);
    double ar, ai, br, bi, cr, ci, dr, di;
    pf_row4_dpp<M>(ar, ai, br, bi, cr, ci, dr, di, wa, wb, wc, wd, ir, ii);
    const double ua = pf_mag<M, SQ>(ar, ai), ub = pf_mag<M, SQ>(br, bi);
    const double uc = pf_mag<M, SQ>(cr, ci), ud = pf_mag<M, SQ>(dr, di);
    f(o, ua);
    f(o + 1, ub);
    f(o + 2, uc);
    f(o + 3, ud);
#pragma unroll
    for (int p = 0; p < P; ++p) {
      wa[p] = na[p];
      wb[p] = nb[p];
      wc[p] = nc[p];
      wd[p] = nd[p];
    }
  }
  // the last n_out - 1 mod 4 rows one at a time (wa, wb, wc hold them)
  if (o < n_out) {
    double ar, ai;
    pf_row1_dpp<M>(ar, ai, wa, ir, ii);
    f(o, pf_mag<M, SQ>(ar, ai));
    ++o;
  }
  if (o < n_out) {
    double ar, ai;
    pf_row1_dpp<M>(ar, ai, wb, ir, ii);
    f(o, pf_mag<M, SQ>(ar, ai));
    ++o;
  }
  if (o < n_out) {
    double ar, ai;
    pf_row1_dpp<M>(ar, ai, wc, ir, ii);
    f(o, pf_mag<M, SQ>(ar, ai));
  }
}

// pf_rows_out's squared magnitudes for the rows of `mask` only (bit r: row r,
// 1 <= r < n_out; wave-uniform), four at a time from the staged rows -- each
// row with pf_row4_dpp's operations, so a row's value is the one pf_rows_out
// gives it.
template <int M, class F>
__device__ __forceinline__ void pf_rows_mask2(const double* s, int n_out, uint64_t mask, const double (&ir)[M],
                                              const double (&ii)[M], F&& f) {
  constexpr int P = PFRow<M>::kPairs;
  if (n_out < 64) mask &= (1ull << n_out) - 1;
  mask &= ~1ull;
  while (mask) {                                     // (uniform)
    int r[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      r[q] = mask ? __builtin_ctzll(mask) : -1;
      mask &= mask - 1;
    }
    double wa[P], wb[P], wc[P], wd[P];
    pf_row_load<M>(s, r[0], wa);
    pf_row_load<M>(s, r[1] < 0 ? r[0] : r[1], wb);
    pf_row_load<M>(s, r[2] < 0 ? r[0] : r[2], wc);
    pf_row_load<M>(s, r[3] < 0 ? r[0] : r[3], wd);
    double ar, ai, br, bi, cr, ci, dr, di;
    pf_row4_dpp<M>(ar, ai, br, bi, cr, ci, dr, di, wa, wb, wc, wd, ir, ii);
    f(r[0], pf_mag<M, false>(ar, ai));
    if (r[1] >= 0) f(r[1], pf_mag<M, false>(br, bi));
    if (r[2] >= 0) f(r[2], pf_mag<M, false>(cr, ci));
    if (r[3] >= 0) f(r[3], pf_mag<M, false>(dr, di));
  }
}

// IO: the storage type of ctrl_p / ctrl_q / v_out (double, or float for
// pgw_pf_solve_f32: inputs widened, every output rounded once; the arithmetic
// is the fp64 solve's).
template <int M, bool UB, bool GC, bool KEEP, class IO = double>
__global__ void __launch_bounds__(kBlock) k_pf_solve(PFArgs a, pgw_pf_tables t, int64_t n,
                                                     const IO* __restrict__ ctrl_p,
                                                     const IO* __restrict__ ctrl_q,
                                                     IO* __restrict__ v_out,
                                                     int32_t* __restrict__ iters) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool valid = e < n;
  long long* const trace = g_pf_trace;
  constexpr bool kKeep = KEEP || !UB || GC;   // general variants always keep the currents
  __shared__ double s_rows[kKeep ? kRowsLds : 1];
  bool rows_lds = false;
  if constexpr (kKeep) rows_lds = pf_rows_stage<M>(t, a.n_out, s_rows);
  // every lane stays to the end of the solve: the DPP broadcasts read all lanes
  PFSolver<M, UB, GC> S;
  S.load(a, t.block);
  pf_trace(trace, 0);                          // (behind the loads: see k_coord_pf)
  double cp[PGW_PF_MAX_CTRL], cq[PGW_PF_MAX_CTRL];
#pragma unroll
  for (int c = 0; c < PGW_PF_MAX_CTRL; ++c) {
    cp[c] = (valid && c < a.n_ctrl && ctrl_p) ? (double)ctrl_p[(int64_t)c * n + e] : 0.0;
    cq[c] = (valid && c < a.n_ctrl && ctrl_q) ? (double)ctrl_q[(int64_t)c * n + e] : 0.0;
  }
  S.powers(a, cp, cq, (t.load_scale && valid) ? t.load_scale[e] : 1.0);
  pf_trace(trace, 1);
  S.template initial<true>(a, t, e, valid);   // (speculative record load: see below)
  pf_trace(trace, 2);
  double v0r, v0i, ir[M], ii[M];
  const int it = S.template iterate<kKeep>(a.max_iter, valid, v0r, v0i, ir, ii);
  pf_trace(trace, 3);
  const int32_t sig = t.sig_out ? S.signature() : 0;
  const double v0 = sqrt(fma(v0i, v0i, v0r * v0r));
  if constexpr (kKeep) __syncthreads();       // the staged rows (every lane is still here)
  pf_trace(trace, 4);
  // element voltages first: they are dead during the output rows
  if (valid && t.U_out) {
#pragma unroll
    for (int k = 0; k < M; ++k) {
      t.U_out[2 * (e * M + k)] = S.ur[k];
      t.U_out[2 * (e * M + k) + 1] = S.ui[k];
    }
  }
  // the output rows with every lane still here (their DPP broadcasts read all
  // lanes); lanes past n store nothing
  double vmn = v0, vmx = v0;      // Python min()/max() over the rows in order
  if constexpr (kKeep) {
    if (v_out || !rows_lds) {
      pf_rows_out<M>(t, rows_lds, s_rows, a.n_out, ir, ii, [&](int o, double v) {
        if (valid && v_out) v_out[(int64_t)o * n + e] = (IO)v;
        vmn = (v < vmn) ? v : vmn;
        vmx = (v > vmx) ? v : vmx;
      });
    } else {
      // extrema only: min / max of |V|^2 over the rows, one sqrt each at the end
      // -- the same values (sqrt is monotone and correctly rounded), without a
      // sqrt per row
      double mn2 = fma(v0i, v0i, v0r * v0r), mx2 = mn2;
      pf_rows_out<M, false>(t, rows_lds, s_rows, a.n_out, ir, ii, [&](int, double m2) {
        mn2 = (m2 < mn2) ? m2 : mn2;
        mx2 = (m2 > mx2) ? m2 : mx2;
      });
      vmn = sqrt(mn2);
      vmx = sqrt(mx2);
    }
  }
  pf_trace(trace, 5);
  if (!valid) return;
  if (t.sig_out) t.sig_out[e] = sig;
  if (a.n_out > 0) {
    if (v_out) v_out[e] = (IO)v0;
    if (t.v_min_out) t.v_min_out[e] = vmn;
    if (t.v_max_out) t.v_max_out[e] = vmx;
  }
  if (iters) iters[e] = it;
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
      bool bad = false;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const double v = ld(act, e, p.act_bld + j);
        bad = bad || oob_bad(v);
        av[j] = p.bld.rescale ? to_raw(v, p.bld.act_low[j], p.bld.act_high[j]) : v;
      }
      if (p.bld.rescale) oob_note(p.bld.oob, bad);
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

// Per-launch constants of the std agent step, derived on the host with the
// same IEEE operations the reference applies (lo + hi, hi - lo), plus the
// reciprocals exact_div needs.
struct StdDerived {
  double act_rng[6], act_sum[6];                  // building actions: hi - lo, hi + lo
  double obs_sum[15], obs_rng[15], obs_rcp[15];   // building obs: lo + hi, hi - lo, 1 / (hi - lo)
  double bat_sum, bat_rng, bat_rcp;               // SoC range
  double rcp_eta_d, rcp_dt_h;                     // storage
};

static StdDerived make_std_derived(const pgw_coord_params& p) {
  StdDerived d = {};
  for (int j = 0; j < 6; ++j) {
    d.act_rng[j] = p.bld.act_high[j] - p.bld.act_low[j];
    d.act_sum[j] = p.bld.act_high[j] + p.bld.act_low[j];
  }
  for (int j = 0; j < 15; ++j) {
    d.obs_sum[j] = p.bld.obs_low[j] + p.bld.obs_high[j];
    d.obs_rng[j] = p.bld.obs_high[j] - p.bld.obs_low[j];
    d.obs_rcp[j] = 1.0 / d.obs_rng[j];
  }
  d.bat_sum = p.bat.soc_min + p.bat.soc_max;
  d.bat_rng = p.bat.soc_max - p.bat.soc_min;
  d.bat_rcp = 1.0 / d.bat_rng;
  d.rcp_eta_d = 1.0 / p.bat.eta_d;
  d.rcp_dt_h = 1.0 / p.bat.dt_h;
  return d;
}

struct StdAgentIn {
  double av[8];     // actions: building 0..5, pv 6, storage 7
  double xs[5];     // building state x_k
  double soc;
};

// Output slots handed to the store callback as soon as they are final.
enum StdSlot { kSlotX = 0, kSlotSoc = 5, kSlotObs = 6, kSlotPower = 23, kSlotReward = 24 };

// One standard agent step for E envs at once (E = 1 or 2, computed stage by
// stage so both envs' chains interleave); every output goes to
// store(slot, v[E]) the moment it is final, so no output stays live.
template <int E, class Store>
__device__ __forceinline__ void std_agent_compute(const pgw_coord_params& p, const StdDerived& dv,
                                                  const pgw_coord_step_info& s, double pv_ob,
                                                  StdAgentIn (&in)[E], Store&& store) {
  const pgw_building_params& B = p.bld;
  double T[E][5], v[E];
  // ---- building
#pragma unroll
  for (int q = 0; q < E; ++q) {
    bool bad = false;
#pragma unroll
    for (int j = 0; j < 6; ++j) {   // to_raw (utils.py:27-43) with host (hi - lo), (hi + lo)
      bad = bad || oob_bad(in[q].av[j]);
      in[q].av[j] = B.rescale ? (clip_fast(in[q].av[j], -1.0, 1.0) * dv.act_rng[j] + dv.act_sum[j]) * 0.5
                              : in[q].av[j];
    }
    if (B.rescale) oob_note(B.oob, bad);
#pragma unroll
    for (int z = 0; z < 5; ++z) T[q][z] = B.C[z] * in[q].xs[z] + B.mean[z];
  }
#pragma unroll
  for (int z = 0; z < 5; ++z) {
    const int nz = z < 2 ? 4 : (z == 2 ? 3 : 2);
#pragma unroll
    for (int q = 0; q < E; ++q) {
      const double u0 = s.ex_t.T_oa - T[q][z];
      const double u1 = in[q].av[z] * (in[q].av[5] - T[q][z]);
      const double u2 = T[q][nz] - T[q][z];
      const double u3 = s.ex_t.q_solar[z];
      double bu = B.B[z][0] * u0;
      bu = bu + B.B[z][1] * u1;
      bu = bu + B.B[z][2] * u2;
      bu = bu + B.B[z][3] * u3;
      in[q].xs[z] = B.A[z] * in[q].xs[z] + bu;   // T[q][*] still holds the pre-step temps
      v[q] = in[q].xs[z];
    }
    store(kSlotX + z, v);
  }
  double pc[E], r_bld[E];
#pragma unroll
  for (int q = 0; q < E; ++q) {
#pragma unroll
    for (int z = 0; z < 5; ++z) T[q][z] = B.C[z] * in[q].xs[z] + B.mean[z];
    pc[q] = building_p_consumed(in[q].av, s.ex_t.T_oa);
    r_bld[q] = building_reward(B, T[q], s.ex_next.comfort_lb, s.ex_next.comfort_ub, pc[q],
                               exact_div(-pc[q], 12.0, 1.0 / 12.0));
  }
  const double lb = s.ex_next.comfort_lb, ub = s.ex_next.comfort_ub;
#pragma unroll
  for (int j = 0; j < 15; ++j) {
#pragma unroll
    for (int q = 0; q < E; ++q) {
      const double o = j < 5 ? T[q][j] - ub : j < 10 ? lb - T[q][j - 5] : j == 10 ? lb
                     : j == 11 ? ub : j == 12 ? s.ex_next.T_oa : j == 13 ? pc[q] : s.ex_next.time_of_day;
      double c = clip_fast(o, B.obs_low[j], B.obs_high[j]);
      if (B.rescale) c = exact_div(2.0 * c - dv.obs_sum[j], dv.obs_rng[j], dv.obs_rcp[j]);
      v[q] = c;
    }
    store(kSlotObs + j, v);
  }
  // ---- pv (obs is env-independent: computed once on the host)
#pragma unroll
  for (int q = 0; q < E; ++q) v[q] = pv_ob;
  store(kSlotObs + 15, v);
  double rp_pv[E], power[E];
#pragma unroll
  for (int q = 0; q < E; ++q) rp_pv[q] = pv_real_power(p.pv, in[q].av[6], s.pv_pmax);
  // ---- storage
#pragma unroll
  for (int q = 0; q < E; ++q) {
    power[q] = battery_step_rcp(p.bat, in[q].av[7], in[q].soc, dv.rcp_eta_d, dv.rcp_dt_h);
    v[q] = in[q].soc;
  }
  store(kSlotSoc, v);
#pragma unroll
  for (int q = 0; q < E; ++q) {
    const double c = clip_fast(in[q].soc, p.bat.soc_min, p.bat.soc_max);
    v[q] = p.bat.rescale ? exact_div(2.0 * c - dv.bat_sum, dv.bat_rng, dv.bat_rcp) : in[q].soc;
  }
  store(kSlotObs + 16, v);
  // MultiComponentEnv sums (base.py:131-137)
#pragma unroll
  for (int q = 0; q < E; ++q) {
    double agent_rp = 0.0;
    agent_rp = agent_rp + pc[q];
    agent_rp = agent_rp + rp_pv[q];
    agent_rp = agent_rp + (-power[q]);
    v[q] = agent_rp;
  }
  store(kSlotPower, v);
#pragma unroll
  for (int q = 0; q < E; ++q) {
    double agent_rew = 0.0;
    agent_rew = agent_rew + r_bld[q];
    agent_rew = agent_rew + 0.0;
    agent_rew = agent_rew + 0.0;
    v[q] = agent_rew;
  }
  store(kSlotReward, v);
}

// Actions are read once per step (a policy's fresh output), so they are
// loaded nontemporally and do not evict the state and agent powers the step
// and the PF kernel re-read: C4 agents 18.0 -> 17.35 us, PF 9.6 -> 9.2 us,
// step 30.4 -> 28.8 us (profiles/r02/act_nt.txt).
template <class S>
__device__ __forceinline__ S ld_act(const S* p) {
  return __builtin_nontemporal_load(p);
}

// Scalar variant: one thread per (env, agent), any action layout.  Bufs =
// pgw_coord_buffers (fp64) or pgw_coord_buffers_f32 (fp32 storage: loads are
// widened, every store rounds the fp64 result once).
template <class Bufs>
__global__ void __launch_bounds__(kBlock) k_coord_agents_std(pgw_coord_params p_,
                                                             pgw_coord_step_info s, int64_t n,
                                                             Bufs b, double pv_ob,
                                                             StdDerived dv) {
  const pgw_coord_params& p = PGW_KERNARG0(pgw_coord_params);   // (no private copy)
  using S = std::remove_pointer_t<decltype(b.soc)>;
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int a = blockIdx.y;
  if (e >= n) return;
  StdAgentIn in[1];
  const S* ap = b.action.ptr + a * b.act_stride_agent + e * b.action.s_env;
#pragma unroll
  for (int j = 0; j < 8; ++j) in[0].av[j] = (double)ld_act(ap + j * b.action.s_dim);
  S* xp = b.x + (int64_t)a * 5 * n + e;
#pragma unroll
  for (int z = 0; z < 5; ++z) in[0].xs[z] = (double)xp[z * n];   // state: cached (re-read next step)
  S* socp = b.soc + (int64_t)a * n + e;
  in[0].soc = (double)*socp;
  S* op = b.obs.ptr + a * b.obs_stride_agent + e * b.obs.s_env;
  std_agent_compute<1>(p, dv, s, pv_ob, in, [&](int slot, const double (&v)[1]) {
    if (slot < kSlotSoc) xp[slot * n] = (S)v[0];
    else if (slot == kSlotSoc) *socp = (S)v[0];
    else if (slot < kSlotPower) st_obs(op + (slot - kSlotObs) * b.obs.s_dim, v[0]);
    else if (slot == kSlotPower) b.agent_power[(int64_t)a * n + e] = (S)v[0];
    else b.reward[(int64_t)a * n + e] = (S)v[0];
  });
}

// Pair variant: one thread per (env pair, agent), every access a 2-vector
// (fp32: 8 B a lane -- the fp64 kernel's request count at half its bytes; with
// one env per lane the fp32 kernel issues as many memory instructions as the
// fp64 one and gains little).  The two envs' chains are computed interleaved
// (std_agent_compute<2>), each exactly as alone.  Needs env-minor action / obs
// views (s_env == 1), an even n and even strides (pairs_ok).
template <class Bufs>
__global__ void __launch_bounds__(kBlock) k_coord_agents_std_x2(pgw_coord_params p_,
                                                                pgw_coord_step_info s, int64_t n,
                                                                Bufs b, double pv_ob, StdDerived dv) {
  const pgw_coord_params& p = PGW_KERNARG0(pgw_coord_params);   // (no private copy)
  using S = std::remove_pointer_t<decltype(b.soc)>;
  typedef S S2 __attribute__((ext_vector_type(2)));
  const int64_t e = 2 * ((int64_t)blockIdx.x * kBlock + threadIdx.x);
  const int a = blockIdx.y;
  if (e >= n) return;
  StdAgentIn in[2];
  const S* ap = b.action.ptr + a * b.act_stride_agent + e;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const S2 v = ld_act(reinterpret_cast<const S2*>(ap + j * b.action.s_dim));
    in[0].av[j] = (double)v.x;
    in[1].av[j] = (double)v.y;
  }
  S* xp = b.x + (int64_t)a * 5 * n + e;
#pragma unroll
  for (int z = 0; z < 5; ++z) {
    const S2 v = *reinterpret_cast<const S2*>(xp + z * n);
    in[0].xs[z] = (double)v.x;
    in[1].xs[z] = (double)v.y;
  }
  S* socp = b.soc + (int64_t)a * n + e;
  {
    const S2 v = *reinterpret_cast<const S2*>(socp);
    in[0].soc = (double)v.x;
    in[1].soc = (double)v.y;
  }
  S* op = b.obs.ptr + a * b.obs_stride_agent + e;
  std_agent_compute<2>(p, dv, s, pv_ob, in, [&](int slot, const double (&v)[2]) {
    const S2 w = {(S)v[0], (S)v[1]};
    if (slot < kSlotSoc) *reinterpret_cast<S2*>(xp + slot * n) = w;
    else if (slot == kSlotSoc) *reinterpret_cast<S2*>(socp) = w;
    else if (slot < kSlotPower)
      __builtin_nontemporal_store(w, reinterpret_cast<S2*>(op + (slot - kSlotObs) * b.obs.s_dim));
    else if (slot == kSlotPower) *reinterpret_cast<S2*>(b.agent_power + (int64_t)a * n + e) = w;
    else *reinterpret_cast<S2*>(b.reward + (int64_t)a * n + e) = w;
  });
}

template <class Bufs>
static bool pairs_ok(const Bufs& b, int64_t n) {
  using S = std::remove_pointer_t<decltype(b.soc)>;
  const auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & (2 * sizeof(S) - 1)) == 0; };
  return n % 2 == 0 && b.action.s_env == 1 && b.obs.s_env == 1 && b.action.s_dim % 2 == 0 &&
         b.obs.s_dim % 2 == 0 && b.act_stride_agent % 2 == 0 && b.obs_stride_agent % 2 == 0 &&
         al(b.action.ptr) && al(b.obs.ptr) && al(b.x) && al(b.soc) && al(b.agent_power) &&
         al(b.reward);
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

// K2: one lane per env -- bus loads (multiagent_env.py:171-181), power flow
// (opendss.py:80-135), CoordinatedMultiBuildingControlEnv.reward_transform
// (train.py:51-63, 71-88) applied to the agent rewards in place.
struct CoordPFArgs {
  int32_t n_agents, coordinated, vv_row;
  int32_t agent_ctrl[PGW_MAX_AGENTS];
  double vv_lo, vv_hi, vv_penalty;
};

// One lane per env (measured alternatives, removed in round 3: 32 envs per
// wave, two lanes per env, and agents + PF in one launch were all slower --
// profiles/r02/pf_half_waves.txt, pf_rows_split_dropped.txt,
// fused_kernel_dropped.txt).
template <int M, bool UB, bool GC, bool KEEP, class Bufs>
__global__ void __launch_bounds__(kBlock) k_coord_pf(CoordPFArgs c, PFArgs a, pgw_pf_tables t,
                                                     int64_t n, Bufs b) {
  using Sto = std::remove_pointer_t<decltype(b.reward)>;   // double, or float (_f32)
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool valid = e < n;
  // read once: a reload per phase would put an L2 round trip on the chain
  long long* const trace = g_pf_trace;
  // HBM first: the agent powers gate the predictor.  The loads are
  // unconditional (clamped indices, then scaled by 1 or 0 -- a select would be
  // sunk back into a branch around the load) so that all of them issue back
  // to back: a load under a branch let the compiler place the first sum right
  // behind it, costing a second HBM round trip.  Lanes past n and agent slots
  // past n_agents are never used.
  double rp[PGW_MAX_AGENTS];
  const int64_t ec = valid ? e : 0;
#pragma unroll
  for (int ag = 0; ag < PGW_MAX_AGENTS; ++ag)
    rp[ag] = (double)b.agent_power[(int64_t)min(ag, c.n_agents - 1) * n + ec] *
             ((valid && ag < c.n_agents) ? 1.0 : 0.0);
  constexpr bool kKeep = KEEP || !UB || GC;   // general variants always keep the currents
  __shared__ double s_rows[kKeep ? kRowsLds : 1];
  bool rows_lds = false;
  if constexpr (kKeep) rows_lds = pf_rows_stage<M>(t, a.n_out, s_rows);
  // every lane stays to the end of the solve: the DPP broadcasts read all lanes
  PFSolver<M, UB, GC> S;
  S.load(a, t.block);
  // phase 0 is stamped once the prologue's loads are in flight: the trace
  // pointer's test waits for its load, which at the kernel's first instruction
  // put a whole dependent L2 round trip ahead of the agent-power loads
  pf_trace(trace, 0);
  double cp[PGW_PF_MAX_CTRL], cq[PGW_PF_MAX_CTRL];
#pragma unroll
  for (int s = 0; s < PGW_PF_MAX_CTRL; ++s) {
    cp[s] = 0.0;
    cq[s] = 0.0;
  }
#pragma unroll
  for (int ag = 0; ag < PGW_MAX_AGENTS; ++ag) {
    const int slot = ag < c.n_agents ? c.agent_ctrl[ag] : -1;
#pragma unroll
    for (int s = 0; s < PGW_PF_MAX_CTRL; ++s) cp[s] = (s == slot) ? cp[s] + rp[ag] : cp[s];
  }
  S.powers(a, cp, cq, 1.0);
  pf_trace(trace, 1);
  S.template initial<!(KEEP || !UB || GC)>(a, t, e, valid);
  pf_trace(trace, 2);
  double v0r, v0i, ir[M], ii[M];
  const int it = S.template iterate<kKeep>(a.max_iter, valid, v0r, v0i, ir, ii);
  pf_trace(trace, 3);
  const double v0 = sqrt(fma(v0i, v0i, v0r * v0r));
  pf_trace(trace, 4);
  if constexpr (kKeep) __syncthreads();       // the staged rows (every lane is still here)
  // the output rows with every lane still here (their DPP broadcasts read all
  // lanes); lanes past n store nothing
  double vsel = v0;
  if constexpr (kKeep)
    pf_rows_out<M>(t, rows_lds, s_rows, a.n_out, ir, ii, [&](int o, double v) {
      if (valid && b.v_out) b.v_out[(int64_t)o * n + e] = (Sto)v;
      vsel = (o == c.vv_row) ? v : vsel;
    });
  if (!valid) return;
  if (b.v_out) b.v_out[e] = (Sto)v0;
  if (b.iters) b.iters[e] = it;
  pf_trace(trace, 5);
  if (c.coordinated) {
    const double vv = pymax(pymax(0.0, c.vv_lo - vsel), vsel - c.vv_hi);
    if (b.vv) b.vv[e] = (Sto)vv;
    const double share = (vv * c.vv_penalty) / (double)c.n_agents;
    // reward -= share as a no-return atomic add of -share: one IEEE add per
    // address (bit-identical to the subtraction, deterministic), no load
    // round trip at the end of the kernel.  fp32 storage: the share is rounded
    // to fp32 first, so the add is RN32(r - RN32(share)).  (Reading the
    // rewards with the powers instead, k_coord_pf_od's form, measured no
    // faster here: profiles/r05/ab_rewx.txt.)
#pragma unroll
    for (int ag = 0; ag < PGW_MAX_AGENTS; ++ag)
      if (ag < c.n_agents)
        (void)__hip_atomic_fetch_add(b.reward + (int64_t)ag * n + e, (Sto)(-share), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ============================================================ OpenDSS snap solve
// (pgw_pf_od, include/pgw.h): the reference's own stopping rule on the fast
// one-lane-per-env kernels.  Per env, from the direct solution u0:
//   iteration 1   u_1 = u1b + P u1P + Q u1Q (the currents at u0 are affine in
//                 the env's controllable P, Q: the host's per-hour table);
//   iteration k   J = I'(u_{k-1}) (compensation currents), u_k = u0 + W'' J --
//                 the resident DPP matvec of the exact solve;
//   test          max over every node of | |V_k| - |V_{k-1}| | <= tol from
//                 iteration min_iter on (Solution.pas Converged).
// Node magnitudes: nodes that are an element's terminal come from |u|; the
// others are check rows V = V0 + G J (LDS-staged, DPP row groups).  Only the
// first n_rep rows are evaluated; the rest are bounded by the last two
// iterations' current changes (pgw.h), and a wave whose bound cannot decide
// some env evaluates them too, in the same iteration -- so the stopping
// iteration is always the exact rule's.  A wave evaluates the rows only in an
// iteration where the element nodes alone do not already fail every env.
struct ODArgs {
  double y0r[PGW_PF_MAX_M], y0i[PGW_PF_MAX_M], esc[PGW_PF_MAX_M];
  double tol, gamma, eps, gmax, gsrc;
  const double* start;
  const double* rows_V0;
  const double* rows_G;
  int32_t min_iter, n_rep, n_rows, max_iter;
  int32_t sparse;                                 // envs a wave's exact test takes one at a time
  int32_t node_mask;                              // bit k: element k is a node (esc[k] > 0)
  const double* resp;                             // response table of the hour (pgw_pf_od.resp) or null
  double resp_x0, resp_inv_h;
  int32_t resp_nseg;
  int32_t resp_v_row;                             // output row of the node records (-1: none)
  const double* resp_v;                           // node records (pgw_pf_od.resp_v) or null
  uint64_t resp_rows;                             // extrema rows of served envs (0: all)
  const double* resp_q;                           // row records (pgw_pf_od.resp_q) or null
  uint64_t resp_q_rows;                           // output rows with a row-record slot (ascending)
  int32_t resp_q_stride, resp_q_k;
};
constexpr int kOdRows = PGW_PF_OD_MAX_ROWS;
constexpr int kOdChunk = 12;                      // check rows per previous-magnitude pass
constexpr int kOdSparse = 4;                      // pgw_pf_od.sparse_envs's default
static_assert(kOdRows <= 32, "od_rows_sparse: one lane pair per row");
// Check-row stride in LDS: the resident row layout plus one pad slot, so that
// od_rows_sparse's lanes (one row each) read 32 rows without bank conflicts.
template <int M> struct ODRow {
  static constexpr int kStride = 16 * PFRow<M>::kPairs + 1;
};
// LDS of the OpenDSS solve, per block of kBlock lanes (one env each):
//   rows  the check rows in the resident row layout (od_row_load), row
//         stride ODRow<M>::kStride
//   st    pgw_pf_od.start (broadcast reads)
//   J     per lane, by iteration parity: iteration k's currents I'(u_{k-1})
//         go to J[k & 1], so the last two iterations' are always there (a lane
//         that stops keeps both: the accepted iteration's are the outputs'
//         input)
//   old   per lane: the previous magnitudes of up to kOdChunk check rows
//         during an exact test
template <int M> struct ODShared {
  double rows[kOdRows * ODRow<M>::kStride];
  double st[12 * M];
  double2 J[2][M * kBlock];
  double old[kOdChunk * kBlock];
};

static ODArgs make_od_args(const pgw_pf_od& d, int max_iter) {
  ODArgs o = {};
  for (int k = 0; k < PGW_PF_MAX_M; ++k) {
    o.y0r[k] = d.y0r[k];
    o.y0i[k] = d.y0i[k];
    o.esc[k] = d.elem_scale[k];
  }
  o.tol = d.tol;
  o.gamma = d.gamma;
  o.eps = d.eps;
  o.gmax = d.gmax;
  o.gsrc = d.gsrc;
  o.start = d.start;
  o.rows_V0 = d.rows_V0;
  o.rows_G = d.rows_G;
  o.min_iter = d.min_iter;
  o.n_rep = d.n_rep;
  o.n_rows = d.n_rows;
  o.max_iter = max_iter;
  o.sparse = d.sparse_envs == 0 ? kOdSparse : d.sparse_envs < 0 ? 0 : min(d.sparse_envs, 64);
  for (int k = 0; k < PGW_PF_MAX_M; ++k)
    if (d.elem_scale[k] > 0.0) o.node_mask |= 1 << k;
  const bool resp = d.resp && d.resp_nseg > 0 && d.resp_h > 0.0;
  o.resp = resp ? d.resp : nullptr;
  o.resp_x0 = d.resp_x0;
  o.resp_inv_h = resp ? 1.0 / d.resp_h : 0.0;
  o.resp_nseg = resp ? d.resp_nseg : 0;
  o.resp_v = (resp && d.resp_v && d.resp_v_row >= 0) ? d.resp_v : nullptr;
  o.resp_v_row = o.resp_v ? d.resp_v_row : -1;
  o.resp_rows = resp ? d.resp_rows : 0;
  const bool q = resp && d.resp_q && d.resp_q_rows != 0 && d.resp_q_stride >= PGW_OD_REC_HEAD + 5 * d.resp_q_k;
  o.resp_q = q ? d.resp_q : nullptr;
  o.resp_q_rows = q ? d.resp_q_rows : 0;
  o.resp_q_stride = q ? d.resp_q_stride : 0;
  o.resp_q_k = q ? d.resp_q_k : 0;
  return o;
}

// NaN-propagating max: an env whose change is NaN never passes the test.
__device__ __forceinline__ double od_max(double a, double b) { return (b > a || b != b) ? b : a; }

// |z| from m2 = |z|^2 for the convergence test: v_rsq_f64 and two Goldschmidt
// steps (~1 ulp for the pu magnitudes here, m2 in [1e-6, 1e6]; 0 for 0) --
// about half the VALU of the IEEE sqrt sequence, which also handles denormals
// and infinities the test never sees.  Every path (fused, generic, fast and
// full row sets) uses it, so they stay bit-identical to each other.
__device__ __forceinline__ double od_mag(double m2) {
  const double r = __builtin_amdgcn_rsq(m2);
  double g = m2 * r, h = 0.5 * r;
  double e = fma(-g, h, 0.5);
  g = fma(g, e, g);
  h = fma(h, e, h);
  const double d = fma(-g, g, m2);
  g = fma(d, h, g);
  return m2 > 0.0 ? g : 0.0;
}

// The check rows (resident row layout) and the first-iteration table into
// LDS, in two halves so that every load of the stage is in flight at once and
// the kernel's own prologue loads go out behind them: od_stage_load issues
// them (a fixed count per lane, no branches: one L2 round trip instead of one
// per 256 entries), od_stage_store writes LDS; the block synchronises before
// use.  (The rolled loop waited for each load before the next: ~5 dependent
// round trips ahead of the solve.)
template <int M> struct ODStage {
  static constexpr int kRowQ = (kOdRows * ODRow<M>::kStride + kBlock - 1) / kBlock;
  static constexpr int kStQ = (12 * M + kBlock - 1) / kBlock;
  double v[kRowQ + kStQ];
  double y0r, y0i, esc;                            // od_solve's resident element constants
};

template <int M>
__device__ __forceinline__ void od_stage_load(const ODArgs& o, const double* start, ODStage<M>& g) {
  constexpr int S = ODRow<M>::kStride;
  const int total = o.n_rows * S;
#pragma unroll
  for (int q = 0; q < ODStage<M>::kRowQ; ++q) {
    const int i = threadIdx.x + q * kBlock;
    const int r = i / S, j = i - r * S;
    // the entry's source; an entry that has none reads row min(r, n_rows - 1),
    // slot min(j, 2M + 1) -- in bounds (the host passes one dummy row when
    // n_rows = 0), so the load may issue unconditionally
    const bool has = i < total && j < 2 + 2 * M;
    const int rc = min(r, max(o.n_rows - 1, 0)), jc = min(j, 1 + 2 * M);
    const double* p = jc < 2 ? o.rows_V0 + (2 * rc + jc)
                             : o.rows_G + (2 * M * rc + (jc < 2 + M ? 2 * (jc - 2) : 2 * (jc - 2 - M) + 1));
    g.v[q] = has ? *p : 0.0;
  }
#pragma unroll
  for (int q = 0; q < ODStage<M>::kStQ; ++q) {
    const int i = threadIdx.x + q * kBlock;
    g.v[ODStage<M>::kRowQ + q] = i < 12 * M ? start[i] : 0.0;
  }
  const int l = threadIdx.x & 15;
  const bool in = l < M;
  g.y0r = in ? o.y0r[l] : 0.0;
  g.y0i = in ? o.y0i[l] : 0.0;
  g.esc = in ? o.esc[l] : 0.0;
}

template <int M>
__device__ __forceinline__ void od_stage_store(const ODArgs& o, const ODStage<M>& g, ODShared<M>& sh) {
  constexpr int S = ODRow<M>::kStride;
  const int total = o.n_rows * S;
#pragma unroll
  for (int q = 0; q < ODStage<M>::kRowQ; ++q) {
    const int i = threadIdx.x + q * kBlock;
    if (i < total) sh.rows[i] = g.v[q];
  }
#pragma unroll
  for (int q = 0; q < ODStage<M>::kStQ; ++q) {
    const int i = threadIdx.x + q * kBlock;
    if (i < 12 * M) sh.st[i] = g.v[ODStage<M>::kRowQ + q];
  }
}

template <int M>
__device__ __forceinline__ void od_row_load(const double* s, int o, double (&w)[PFRow<M>::kPairs]) {
  const double* r = s + ODRow<M>::kStride * o + (threadIdx.x & 15);
#pragma unroll
  for (int p = 0; p < PFRow<M>::kPairs; ++p) w[p] = r[16 * p];
}

// Rows [r0, r1) (r1 - r0 <= kOdChunk) from the currents in J (the lane's
// slots).  CMP = false: their magnitudes into old[r - r0].  CMP = true:
// err <- max | |V_r| - old |, amin <- min old.  Four rows per DPP group, the
// next group's operands loaded while this one computes; every lane runs it
// (the broadcasts read all lanes).
template <int M, bool CMP>
__device__ __forceinline__ void od_rows(const ODShared<M>& sh, const double2* J, double* old, int r0, int r1,
                                        double& err, double& amin) {
  constexpr int P = PFRow<M>::kPairs;
  const int tid = threadIdx.x;
  const int last = r1 - 1;
  double ir[M], ii[M];
#pragma unroll
  for (int k = 0; k < M; ++k) {
    const double2 j = J[k * kBlock + tid];
    ir[k] = j.x;
    ii[k] = j.y;
  }
  double wa[P], wb[P], wc[P], wd[P];
  od_row_load<M>(sh.rows, r0, wa);
  od_row_load<M>(sh.rows, min(r0 + 1, last), wb);
  od_row_load<M>(sh.rows, min(r0 + 2, last), wc);
  od_row_load<M>(sh.rows, min(r0 + 3, last), wd);
  for (int o = r0; o < r1; o += 4) {
    double na[P], nb[P], nc[P], nd[P];
    od_row_load<M>(sh.rows, min(o + 4, last), na);     // the next group in flight
    od_row_load<M>(sh.rows, min(o + 5, last), nb);
    od_row_load<M>(sh.rows, min(o + 6, last), nc);
    od_row_load<M>(sh.rows, min(o + 7, last), nd);
    double* const ol = old + (o - r0) * kBlock + tid;
    double om[4];
    if constexpr (CMP) {
#pragma unroll
      for (int q = 0; q < 4; ++q) om[q] = ol[min(q, last - o) * kBlock];
    }
    __builtin_amdgcn_sched_barrier(0);
    double ar, ai, br, bi, cr, ci, dr, di;
    pf_row4_dpp<M>(ar, ai, br, bi, cr, ci, dr, di, wa, wb, wc, wd, ir, ii);
    const double mg[4] = {od_mag(fma(ai, ai, ar * ar)), od_mag(fma(bi, bi, br * br)),
                          od_mag(fma(ci, ci, cr * cr)), od_mag(fma(di, di, dr * dr))};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (o + q < r1) {                                 // (uniform)
        if constexpr (CMP) {
          err = od_max(err, fabs(mg[q] - om[q]));
          amin = fmin(amin, om[q]);
        } else {
          ol[q * kBlock] = mg[q];
        }
      }
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
      wa[p] = na[p];
      wb[p] = nb[p];
      wc[p] = nc[p];
      wd[p] = nd[p];
    }
  }
}

// Rows [r0, r1) of an exact test: previous magnitudes from the previous
// iteration's currents, new ones from this iteration's, kOdChunk rows at a time.
template <int M>
__device__ __forceinline__ void od_check_rows(ODShared<M>& sh, const double2* cur, const double2* prv, int r0,
                                              int r1, double& err, double& amin) {
  for (int c = r0; c < r1; c += kOdChunk) {            // (uniform)
    const int e = min(c + kOdChunk, r1);
    od_rows<M, false>(sh, prv, sh.old, c, e, err, amin);
    od_rows<M, true>(sh, cur, sh.old, c, e, err, amin);
  }
}

// Rows [r0, r1) (<= 32) of an exact test for the few envs of the wave in
// `envs` (lane bits), one env at a time, transposed: lane 2 q evaluates row
// r0 + q from the env's previous currents, lane 2 q + 1 from its current ones
// -- each with pf_node_pu's operations in od_rows's order, so the magnitudes
// are bit-identical --, and a butterfly reduces the row changes and previous
// magnitudes onto the env's lane.  For a wave where one env or a few need the
// test, instead of every lane's DPP row groups.
template <int M>
__device__ __forceinline__ void od_rows_sparse(const ODShared<M>& sh, const double2* cur, const double2* prv,
                                               int r0, int r1, uint64_t envs, double& err, double& amin) {
  if (r0 >= r1) return;                              // (uniform)
  const int lane = threadIdx.x & 63;
  const int row = min(r0 + (lane >> 1), r1 - 1);
  const bool on = r0 + (lane >> 1) < r1;
  const double* R = sh.rows + ODRow<M>::kStride * row;
  const double2* J = (lane & 1) ? cur : prv;
  const int wave0 = threadIdx.x & ~63;
  while (envs) {                                     // (uniform)
    const int L = __builtin_ctzll(envs);
    envs &= envs - 1;
    const double2* Je = J + wave0 + L;
    double vr = R[0], vi = R[1];
#pragma unroll
    for (int k = 0; k < M; ++k) {
      const double gr = R[2 + k], gi = R[2 + M + k];
      const double2 j = Je[k * kBlock];
      vr = fma(gr, j.x, vr);
      vi = fma(gr, j.y, vi);
      vr = fma(-gi, j.y, vr);
      vi = fma(gi, j.x, vi);
    }
    const double mg = od_mag(fma(vi, vi, vr * vr));
    const double mn = __shfl_xor(mg, 1);             // even lanes: the new magnitude
    const bool prev_lane = on && !(lane & 1);
    double we = prev_lane ? fabs(mn - mg) : 0.0;
    double wa = prev_lane ? mg : __builtin_huge_val();
#pragma unroll
    for (int x = 1; x < 64; x <<= 1) {
      we = od_max(we, __shfl_xor(we, x));
      wa = fmin(wa, __shfl_xor(wa, x));
    }
    if (lane == L) {
      err = od_max(err, we);
      amin = fmin(amin, wa);
    }
  }
}

// The env's test after an iteration: lo = the exact changes (element nodes
// and the evaluated rows), hi = lo plus the bounds of the unevaluated rows.
// Returns 1 converged, 0 not, -1 undecided (the bounds straddle tol).
template <class OA>
__device__ __forceinline__ int od_decide(const OA& o, bool full, int it, double lo, double amin,
                                         double dsum, double jsum) {
  if (it < o.min_iter || lo > o.tol || lo != lo) return 0;
  if (full) return lo <= o.tol ? 1 : 0;
  const double d = o.gmax * dsum;                       // >= |dV| of any evaluated node
  if (!(amin - d > 0.0)) return -1;
  // members: err_j <= err_r + |d_j - d_r| + 2 |V_j - V_r| |d_r| / (|V_r| - |d_r|)
  const double delta = o.gamma * dsum + 2.0 * (o.eps + o.gamma * jsum) * d / (amin - d);
  const double hi = fmax(lo + delta, o.gsrc * dsum);   // source side: err_j <= |d_j|
  return hi <= o.tol ? 1 : -1;
}

// The currents of the accepted iteration `it` (od_solve's return).
template <int M>
__device__ __forceinline__ void od_load_J(const ODShared<M>& sh, int it, double (&ir)[M], double (&ii)[M]) {
  const double2* J = sh.J[abs(it) & 1];
#pragma unroll
  for (int k = 0; k < M; ++k) {
    const double2 j = J[k * kBlock + threadIdx.x];
    ir[k] = j.x;
    ii[k] = j.y;
  }
}

// The whole snap solve of the lane's env (S: block, powers loaded; sh staged
// and synchronised; min_iter >= 2, check_od).  Returns the iteration count,
// negative when stopped by max_iter; the accepted currents are in
// sh.J[|count| & 1].
//   iteration 1  u_1 from the affine table; no test (it < min_iter).
//   iteration k  currents and matvec; then, without a square root, a lower
//                bound of every element node's change (|a| + |b| <= (a^2 +
//                b^2)/2 + 1): above tol for some node means not converged,
//                exactly.  Only when some lane of the wave is left (k >=
//                min_iter, no node above tol) does the wave run the exact test:
//                element nodes, then the rows' previous magnitudes from the
//                previous currents and the new ones from this iteration's --
//                the first n_rep rows, the bounded ones only when some env's
//                bounds cannot decide (it then takes the exact decision).
// SIG (the response-table builder, pgw_pf_od_probe): *sig accumulates, per
// iteration the env runs, the load band of every element of the iterate whose
// currents it forms (u_1 .. u_{k*-1}), then the returned count: a 64-bit FNV-1a
// style hash that tells the smooth pieces of the solve as a function of P apart.
constexpr uint64_t kFnvBasis = 0xcbf29ce484222325ull, kFnvPrime = 0x100000001b3ull;
template <int M, bool SIG = false>
__device__ int od_solve(PFSolver<M, true, false>& S, const ODArgs& o, const ODStage<M>& g, bool valid,
                        ODShared<M>& sh, uint64_t* sig = nullptr) {
  static_assert(kOdRows <= 2 * M, "od_rows keeps two row magnitudes per current slot");
  const int tid = threadIdx.x;
  // per-element constants resident for DPP: y0' (re, im) and the node scale
  // (loaded with the stage)
  double yres[2] = {g.y0r, g.y0i};
  const double eres = g.esc;
  // |a| - |b| > tol for sure when |a^2 - b^2| > tol_lo ((a^2 + b^2)/2 + 1)
  const double tol_lo = o.tol * (1.0 + 0x1p-30);
  const bool bounded = o.n_rep < o.n_rows;
  // ---- iteration 1 from the affine tables: u_1 now; its currents I'(u0)
  // (an exact test's previous ones at iteration 2, or the outputs when
  // max_iter = 1) only when needed
  const double* st = sh.st;
  auto affine = [&](int c, double& re, double& im) {    // table entry c (of 3 M)
    re = fma(S.qc, st[2 * (2 * M + c)], fma(S.pc, st[2 * (M + c)], st[2 * c]));
    im = fma(S.qc, st[2 * (2 * M + c) + 1], fma(S.pc, st[2 * (M + c) + 1], st[2 * c + 1]));
  };
  auto currents_1 = [&]() {
#pragma unroll
    for (int k = 0; k < M; ++k) {
      double jr, ji;
      affine(3 * M + k, jr, ji);
      sh.J[1][k * kBlock + tid] = make_double2(jr, ji);
    }
  };
#pragma unroll
  for (int k = 0; k < M; ++k) affine(k, S.ur[k], S.ui[k]);
  if (o.max_iter <= 1) currents_1();                 // (uniform)
  int it = 1, my_it = 1;
  bool done = !valid || o.max_iter <= 1, conv_ok = !valid;
  while (__ballot(!done) != 0ull) {
    ++it;
    double2* const cur = sh.J[it & 1];
    const double2* const prv = sh.J[(it & 1) ^ 1];
    if constexpr (SIG) {
      uint64_t bands = 0;
      static_for<0, M>([&](auto kk) {
        constexpr int k = decltype(kk)::value;
        const double m2 = fma(S.ui[k], S.ui[k], S.ur[k] * S.ur[k]);     // (current_od's)
        const uint64_t b = (uint64_t)(m2 > S.lo2) + (uint64_t)(m2 > S.mn2) + (uint64_t)(m2 > S.mx2);
        bands |= b << (2 * k);
      });
      if (!done) *sig = (*sig ^ bands) * kFnvPrime;
    }
    // ---- currents of u_{k-1} (into LDS), u_k by the matvec.  (Interleaving
    // element k+1's current law between slices of column k's FMAs measured no
    // faster -- profiles/r04/ab_pipelined_column_loop.txt: the wave is bound by
    // its DPP issue rate, not by the chain's latency.)
    double A[M], Bs[M], C[M];
    pf_acc_init<M>(A, C, S.w);
#pragma unroll
    for (int i = 0; i < M; ++i) Bs[i] = 0.0;
    auto column = [&](auto kk, double ir, double ii) {
      constexpr int k = decltype(kk)::value;
      pf_column<M, k>(A, Bs, C, S.w, ir, ii, ir + ii);
      if (!done) cur[k * kBlock + tid] = make_double2(ir, ii);
    };
    static_for<0, M / 2>([&](auto h) {
      constexpr int k0 = 2 * h, k1 = 2 * h + 1;
      double ir0, ii0, ir1, ii1, y0r0, y0i0, y0r1, y0i1;
      pf_od_elem<M, k0>(y0r0, y0i0, yres);
      pf_od_elem<M, k1>(y0r1, y0i1, yres);
      S.template current_od<k0>(y0r0, y0i0, ir0, ii0);
      S.template current_od<k1>(y0r1, y0i1, ir1, ii1);
      column(std::integral_constant<int, k0>{}, ir0, ii0);
      column(std::integral_constant<int, k1>{}, ir1, ii1);
    });
    if constexpr (M % 2) {
      double ir, ii, y0r, y0i;
      pf_od_elem<M, M - 1>(y0r, y0i, yres);
      S.template current_od<M - 1>(y0r, y0i, ir, ii);
      column(std::integral_constant<int, M - 1>{}, ir, ii);
    }
    double nr[M], ni[M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      nr[i] = A[i] - Bs[i];
      ni[i] = (C[i] - A[i]) - Bs[i];
    }
    // ---- the square-root-free lower bound over the element nodes
    bool hit = false;
    static_for<0, M>([&](auto kk) {
      constexpr int i = decltype(kk)::value;
      if ((o.node_mask >> i) & 1) {                   // (uniform) the element is a node
        const double e = pf_bc16<i % 16>(eres), e2 = e * e;
        const double a2 = fma(ni[i], ni[i], nr[i] * nr[i]) * e2;
        const double b2 = fma(S.ui[i], S.ui[i], S.ur[i] * S.ur[i]) * e2;
        hit = hit || fabs(a2 - b2) > tol_lo * fma(0.5, a2 + b2, 1.0);
      }
    });
    const bool need = !done && it >= o.min_iter && !hit;
    const uint64_t needs = __ballot(need);
    const bool exact = needs != 0ull;                 // (uniform)
    double err = 0.0, amin = __builtin_huge_val();
    if (exact) {
      static_for<0, M>([&](auto kk) {
        constexpr int i = decltype(kk)::value;
        if ((o.node_mask >> i) & 1) {                 // (uniform)
          const double e = pf_bc16<i % 16>(eres);
          const double mo = od_mag(fma(S.ui[i], S.ui[i], S.ur[i] * S.ur[i])) * e;
          const double mn = od_mag(fma(ni[i], ni[i], nr[i] * nr[i])) * e;
          err = od_max(err, fabs(mn - mo));
          amin = fmin(amin, mo);
        }
      });
    }
#pragma unroll
    for (int i = 0; i < M; ++i) {
      S.ur[i] = done ? S.ur[i] : nr[i];
      S.ui[i] = done ? S.ui[i] : ni[i];
    }
    int d = 0;
    if (exact) {
      if (it == 2) currents_1();                     // (uniform)
      // the change bound's sums: this iteration's currents against the
      // previous ones (the rounding, ~1e-15 relative, as slack)
      double dsum = 0.0, jsum = 0.0;
#pragma unroll
      for (int k = 0; k < M; ++k) {
        const double2 c = cur[k * kBlock + tid], p = prv[k * kBlock + tid];
        dsum += fabs(c.x - p.x) + fabs(c.y - p.y);
        jsum += fabs(p.x) + fabs(p.y);
      }
      dsum = fma(0x1p-40, jsum + dsum, dsum);
      jsum = fma(0x1p-40, jsum, jsum);
      // (an env that is not tested here already fails at an element node
      // or is below min_iter: its decision does not read the rows)
      // od_rows_sparse reads other lanes' current slots written above in this
      // iteration: make the cross-lane LDS dependency explicit
      __builtin_amdgcn_wave_barrier();
      if (__popcll(needs) <= o.sparse) od_rows_sparse<M>(sh, cur, prv, 0, o.n_rep, needs, err, amin);
      else od_check_rows<M>(sh, cur, prv, 0, o.n_rep, err, amin);
      d = od_decide(o, !bounded, it, err, amin, dsum, jsum);
      // an env whose bounds cannot decide: its wave evaluates the bounded
      // rows too, in this iteration, and the env takes the exact decision
      const uint64_t undecided = __ballot(!done && d < 0);
      if (undecided != 0ull) {
        if (__popcll(undecided) <= o.sparse)
          od_rows_sparse<M>(sh, cur, prv, o.n_rep, o.n_rows, undecided, err, amin);
        else
          od_check_rows<M>(sh, cur, prv, o.n_rep, o.n_rows, err, amin);
        d = d < 0 ? od_decide(o, true, it, err, amin, dsum, jsum) : d;
      }
    }
    my_it = done ? my_it : it;
    conv_ok = conv_ok || (!done && d > 0);
    done = done || d > 0 || it >= o.max_iter;
  }
  const int ret = conv_ok ? my_it : -my_it;
  if constexpr (SIG) *sig = (*sig ^ (uint64_t)(uint32_t)ret) * kFnvPrime;
  return ret;
}

// ---- the response table (pgw_pf_od.resp) ---------------------------------
// Record r (PGW_OD_REC doubles, 16-byte aligned): as double2, [0] (lo, hi),
// [1] (xc, inv_hw), [2] (k* | next << 32, -), then c0, c1, c2 per element.
constexpr int kOdHops = 8;                         // records tried per env (chain length)
__device__ __forceinline__ void od_rec_meta(double v, int& it, int& next) {
  const long long b = __double_as_longlong(v);
  it = (int)(uint32_t)(b & 0xffffffffll);
  next = (int)(b >> 32);
}
// J'_k at t = (P - xc) inv_hw: c0 + t (c1 + t c2) -- the step kernels and
// pgw_pf_od_resp_check evaluate it with these operations.
__device__ __forceinline__ double2 od_rec_j(double2 c0, double2 c1, double2 c2, double t) {
  return make_double2(fma(t, fma(t, c2.x, c1.x), c0.x), fma(t, fma(t, c2.y, c1.y), c0.y));
}
// The env's currents J' and iteration count from the table: false when P
// (with Q = 0) lies in no piece -- then the env runs the snap solve.
template <int M>
__device__ __forceinline__ bool od_resp_lookup(const ODArgs& o, double P, double Q, double (&jr)[M],
                                               double (&ji)[M], int& it, double2& vf, int& rec, double& tq) {
  constexpr int R2 = PGW_OD_REC(M) / 2;
  const double g = (P - o.resp_x0) * o.resp_inv_h;
  if (!(Q == 0.0) || !(g >= 0.0 && g < (double)o.resp_nseg)) return false;
  int r = (int)g;
  for (int hop = 0; hop < kOdHops; ++hop) {
    const double2* rp = reinterpret_cast<const double2*>(o.resp) + (int64_t)r * R2;
    double2 c[3 * M];
    const double2 h0 = rp[0], h1 = rp[1], h2 = rp[2];
#pragma unroll
    for (int q = 0; q < 3 * M; ++q) c[q] = rp[3 + q];       // in flight with the header
    // the node record's coefficients in the same round trip (its header is a
    // copy of this one); zero without node records
    double2 v0 = make_double2(0.0, 0.0), v1 = v0, v2 = v0;
    if (o.resp_v) {
      const double2* vr = reinterpret_cast<const double2*>(o.resp_v) + (int64_t)r * (PGW_OD_VREC / 2);
      v0 = vr[3];
      v1 = vr[4];
      v2 = vr[5];
    }
    int k_it, next;
    od_rec_meta(h2.x, k_it, next);
    if (P >= h0.x && P <= h0.y) {
      if (k_it == 0) return false;                          // a piece without a fit
      const double t = (P - h1.x) * h1.y;
#pragma unroll
      for (int k = 0; k < M; ++k) {
        const double2 j = od_rec_j(c[k], c[M + k], c[2 * M + k], t);
        jr[k] = j.x;
        ji[k] = j.y;
      }
      it = k_it;
      vf = od_rec_j(v0, v1, v2, t);
      rec = r;
      tq = t;
      return true;
    }
    if (next < 0) return false;
    r = next;
  }
  return false;
}

// ---- row records (pgw_pf_od.resp_q): per response record, the squared
// magnitude of each listed output row as a quartic in the record's t,
// |V0 + G J'(t)|^2 = a0 + t (a1 + t (a2 + t (a3 + t a4))), composed on the
// host from the same pieces.  A served env takes every listed row's value from
// them on every path (all rows, extrema only, fused), so each row is the same
// bit for bit whichever kernel and row set computes it; an extrema-only solve
// whose block the table serves entirely reads only these records.
__device__ __forceinline__ int od_q_slot(const ODArgs& o, int ro) {
  if (!o.resp_q || ro < 0 || ro >= 64 || !((o.resp_q_rows >> ro) & 1ull)) return -1;
  return __popcll(o.resp_q_rows & ((1ull << ro) - 1ull));
}
__device__ __forceinline__ double od_q_m2(const ODArgs& o, int rec, int slot, double t) {
  const double* q = o.resp_q + (int64_t)rec * o.resp_q_stride + PGW_OD_REC_HEAD + 5 * slot;
  return fma(t, fma(t, fma(t, fma(t, q[4], q[3]), q[2]), q[1]), q[0]);
}
// A record's candidate slots: header word 5 of its row record, the slots the
// host proved can hold the extremum of an env the record serves
// (OpenDSSSolver._od_qrows; 0: every slot).
__device__ __forceinline__ uint64_t od_q_cand(double h5) {
  const uint64_t m = (uint64_t)__double_as_longlong(h5);
  return m ? m : ~0ull;
}
// The piece of P (Q = 0) from the row records' headers alone (the chain of
// od_resp_lookup, same decisions): record index, t, the count and the
// record's candidate slots.
__device__ __forceinline__ bool od_q_find(const ODArgs& o, double P, double Q, int& it, int& rec, double& tq,
                                          uint64_t& qm) {
  const double g = (P - o.resp_x0) * o.resp_inv_h;
  if (!(Q == 0.0) || !(g >= 0.0 && g < (double)o.resp_nseg)) return false;
  int r = (int)g;
  for (int hop = 0; hop < kOdHops; ++hop) {
    const double2* h = reinterpret_cast<const double2*>(o.resp_q + (int64_t)r * o.resp_q_stride);
    const double2 h0 = h[0], h1 = h[1], h2 = h[2];
    int k_it, next;
    od_rec_meta(h2.x, k_it, next);
    if (P >= h0.x && P <= h0.y) {
      if (k_it == 0) return false;
      it = k_it;
      rec = r;
      tq = (P - h1.x) * h1.y;
      qm = od_q_cand(h2.y);
      return true;
    }
    if (next < 0) return false;
    r = next;
  }
  return false;
}
// Record rec's currents J'(t) (od_resp_lookup's values) and node-record value.
template <int M>
__device__ __forceinline__ void od_resp_at(const ODArgs& o, int rec, double t, double (&jr)[M], double (&ji)[M],
                                           double2& vf) {
  constexpr int R2 = PGW_OD_REC(M) / 2;
  const double2* rp = reinterpret_cast<const double2*>(o.resp) + (int64_t)rec * R2;
#pragma unroll
  for (int k = 0; k < M; ++k) {
    const double2 j = od_rec_j(rp[3 + k], rp[3 + M + k], rp[3 + 2 * M + k], t);
    jr[k] = j.x;
    ji[k] = j.y;
  }
  if (o.resp_v) {
    const double2* vr = reinterpret_cast<const double2*>(o.resp_v) + (int64_t)rec * (PGW_OD_VREC / 2);
    vf = od_rec_j(vr[3], vr[4], vr[5], t);
  }
}

// od_resp_lookup for a solve whose only output is the node records' row: the
// 96-byte node records alone (their headers decide exactly as the response
// records', so the same envs are served, with the same counts).
template <class OA>
__device__ __forceinline__ bool od_resp_lookup_v(const OA& o, double P, double Q, double2& v, int& it) {
  constexpr int R2 = PGW_OD_VREC / 2;
  const double g = (P - o.resp_x0) * o.resp_inv_h;
  if (!(Q == 0.0) || !(g >= 0.0 && g < (double)o.resp_nseg)) return false;
  int r = (int)g;
  for (int hop = 0; hop < kOdHops; ++hop) {
    const double2* rec = reinterpret_cast<const double2*>(o.resp_v) + (int64_t)r * R2;
    const double2 h0 = rec[0], h1 = rec[1], h2 = rec[2], c0 = rec[3], c1 = rec[4], c2 = rec[5];
    int k_it, next;
    od_rec_meta(h2.x, k_it, next);
    if (P >= h0.x && P <= h0.y) {
      if (k_it == 0) return false;
      v = od_rec_j(c0, c1, c2, (P - h1.x) * h1.y);
      it = k_it;
      return true;
    }
    if (next < 0) return false;
    r = next;
  }
  return false;
}

// The envs of the block the table does not cover: stage the check rows (the
// stage loads already issued unless `late`) and run the snap solve for them;
// their currents and counts replace (jr, ji, it).  The other lanes park their
// table currents in their own sh.J[0] slots through the solve (a lane that does
// not solve never writes its slots there: od_solve stores currents only while
// the env runs, and currents_1 writes sh.J[1]), so the solve's registers do
// not add to them.  Block-uniform barriers: every lane of the block calls it.
template <int M>
__device__ __forceinline__ void od_fallback(PFSolver<M, true, false>& S, const ODArgs& o, const double* start,
                                            ODStage<M>& stg, bool late, ODShared<M>& sh, bool need,
                                            double (&jr)[M], double (&ji)[M], int& it) {
  if (!__syncthreads_or(need)) return;               // (block-uniform)
  const int tid = threadIdx.x;
  if (!need) {
#pragma unroll
    for (int k = 0; k < M; ++k) sh.J[0][k * kBlock + tid] = make_double2(jr[k], ji[k]);
  }
  if (late) od_stage_load<M>(o, start, stg);
  od_stage_store<M>(o, stg, sh);
  __syncthreads();                                   // the staged check rows
  int its = 0;
  if (__ballot(need) != 0ull)                        // (wave-uniform) some env of this wave
    its = od_solve<M>(S, o, stg, need, sh);
  const double2* J = need ? sh.J[abs(its) & 1] : sh.J[0];
#pragma unroll
  for (int k = 0; k < M; ++k) {
    const double2 j = J[k * kBlock + tid];
    jr[k] = j.x;
    ji[k] = j.y;
  }
  it = need ? its : it;
}

// Output rows 1.. of the OpenDSS-rule kernels, staged in the LDS the solve
// leaves idle once the block is past it: od_rows_issue loads a row entry per
// lane and slot (a fixed count, clamped in-bounds addresses, all in flight
// with the prologue's loads), od_rows_put stores them in pf_rows_out's resident
// row layout, whose DPP row groups then evaluate the rows (the exact kernels'
// path; per row pf_node_pu's operations, so every node is bit-identical
// whichever kernel and row computes it).
constexpr int kOdRowQ = kRowsLds / kBlock;
template <int M>
__device__ __forceinline__ bool od_rows_lds(int n_out) {
  return n_out > 1 && n_out * 16 * PFRow<M>::kPairs <= kRowsLds;
}
template <int M>
__device__ __forceinline__ void od_rows_issue(const pgw_pf_tables& t, int n_out, double (&v)[kOdRowQ]) {
  constexpr int S = 16 * PFRow<M>::kPairs;
  const int total = n_out * S;
#pragma unroll
  for (int q = 0; q < kOdRowQ; ++q) {
    const int i = threadIdx.x + q * kBlock;
    const int o = i / S, j = i - o * S;
    const bool has = i < total && j < 2 + 2 * M;
    const int oc = min(o, max(n_out - 1, 0)), jc = min(j, 1 + 2 * M);
    const double* p = jc < 2 ? t.V0 + (2 * oc + jc)
                             : t.G + (2 * M * oc + (jc < 2 + M ? 2 * (jc - 2) : 2 * (jc - 2 - M) + 1));
    v[q] = has ? *p : 0.0;
  }
}
template <int M>
__device__ __forceinline__ double* od_rows_put(ODShared<M>& sh, int n_out, const double (&v)[kOdRowQ]) {
  static_assert(sizeof(ODShared<M>) >= kRowsLds * sizeof(double), "the rows fit the solve's LDS");
  constexpr int S = 16 * PFRow<M>::kPairs;
  double* s = reinterpret_cast<double*>(&sh);
  __syncthreads();                                   // every lane past the solve (and its sh.J reads)
#pragma unroll
  for (int q = 0; q < kOdRowQ; ++q) {
    const int i = threadIdx.x + q * kBlock;
    if (i < n_out * S) s[i] = v[q];
  }
  __syncthreads();
  return s;
}

// Fused C4 step, OpenDSS rule: k_coord_pf's prologue (agent powers -> bus
// load) and epilogue (output row 0 = the coordinated bus, violation, reward),
// the snap solve in between.
// TR: the trace instantiation (pgw_debug_pf_trace set): phase stamps 0 entry,
// 1 powers summed, 2 table lookup done, 3 past the fallback, 4 node 0, 5 rows,
// 6 reward atomics issued.
// LIST (k_coord_pf_od_list): env e comes from the fused step's list of envs
// the table did not serve (k_coord_step_od), so every valid lane solves; the
// agents' rewards it reads are their raw values, which k_coord_step_od left
// in place for exactly these envs.
template <int M, class Bufs, bool TR, bool LIST>
__device__ __forceinline__ void coord_pf_od_env(const CoordPFArgs& c, const PFArgs& a, const ODArgs& o,
                                                const pgw_pf_tables& t, int64_t n, const Bufs& b, int64_t e,
                                                bool valid, ODShared<M>& sh) {
  using Sto = std::remove_pointer_t<decltype(b.reward)>;
  long long* const tr = TR ? g_pf_trace : nullptr;
  if constexpr (TR) pf_trace(tr, 0);
  ODStage<M> stg;
  // without a response table every env solves: the stage loads go out first,
  // in flight with the loads below; with one only a block that needs them does
  const bool early = LIST || o.resp == nullptr;
  if (early) od_stage_load<M>(o, o.start, stg);
  const bool rows_lds = od_rows_lds<M>(a.n_out);     // (uniform) a history slot: every node
  double rv[kOdRowQ];
  if (rows_lds) od_rows_issue<M>(t, a.n_out, rv);
  double rp[PGW_MAX_AGENTS];
  const int64_t ec = valid ? e : 0;
#pragma unroll
  for (int ag = 0; ag < PGW_MAX_AGENTS; ++ag)
    rp[ag] = (double)b.agent_power[(int64_t)min(ag, c.n_agents - 1) * n + ec] *
             ((valid && ag < c.n_agents) ? 1.0 : 0.0);
  // the agents' rewards, read with their powers (one round trip): the
  // epilogue stores reward + (-share) -- the read-modify-write's value --
  // instead of 5 device-scope atomics at the end
  Sto rw[PGW_MAX_AGENTS];
#pragma unroll
  for (int ag = 0; ag < PGW_MAX_AGENTS; ++ag)
    rw[ag] = (c.coordinated && ag < c.n_agents) ? b.reward[(int64_t)ag * n + ec] : (Sto)0;
  // with node records for output row 0 and no other row (the fused C4 step),
  // the 96-byte node record is all a served env reads
  const bool vonly = o.resp_v != nullptr && o.resp_v_row == 0 && a.n_out == 1;   // (uniform)
  // ... and the solve's operands (the resident block) only a wave with an env
  // the table left needs: there they go out after the lookup
  const bool lazy = vonly && !LIST && o.resp != nullptr;                          // (uniform)
  PFSolver<M, true, false> S;
  if (!lazy) S.load(a, t.block);
  double cp[PGW_PF_MAX_CTRL], cq[PGW_PF_MAX_CTRL];
#pragma unroll
  for (int s = 0; s < PGW_PF_MAX_CTRL; ++s) {
    cp[s] = 0.0;
    cq[s] = 0.0;
  }
#pragma unroll
  for (int ag = 0; ag < PGW_MAX_AGENTS; ++ag) {
    const int slot = ag < c.n_agents ? c.agent_ctrl[ag] : -1;
#pragma unroll
    for (int s = 0; s < PGW_PF_MAX_CTRL; ++s) cp[s] = (s == slot) ? cp[s] + rp[ag] : cp[s];
  }
  S.powers(a, cp, cq, 1.0);
  if constexpr (TR) { if (S.pc != -1e300) pf_trace(tr, 1); }
  double ir[M], ii[M], v0r = 0.0, v0i = 0.0;
#pragma unroll
  for (int k = 0; k < M; ++k) ir[k] = ii[k] = 0.0;
  int it = 0;
  double2 vf = make_double2(0.0, 0.0);
  int rec = 0;
  double tq = 0.0;
  bool served;
  if constexpr (LIST) {
    served = false;
  } else if (vonly) {
    served = valid && od_resp_lookup_v(o, S.pc, S.qc, vf, it);
  } else {
    served = valid && o.resp && od_resp_lookup<M>(o, S.pc, S.qc, ir, ii, it, vf, rec, tq);
  }
  const bool need = valid && !served;
  if (lazy && __ballot(need) != 0ull) S.load(a, t.block);   // (wave-uniform)
  if constexpr (TR) { if (ir[0] != -1e300 && vf.x != -1e300) pf_trace(tr, 2); }
  od_fallback<M>(S, o, o.start, stg, !early, sh, need, ir, ii, it);
  if constexpr (TR) pf_trace(tr, 3);
  // node 0 from the currents -- unless every env of the wave takes it from its
  // node record anyway (the fused C4 step's usual case; pf_node0's DPP sums
  // need the whole wave, so the test is wave-uniform)
  if (!(vonly && __ballot(valid && !served) == 0ull)) pf_node0<M>(v0r, v0i, S.w, ir, ii);
  if (served && o.resp_v_row == 0) {                 // the node record's row
    v0r = vf.x;
    v0i = vf.y;
  }
  double m2_0 = fma(v0i, v0i, v0r * v0r);
  if (o.resp_q) {                                    // (uniform) the row records' row 0
    const int q0 = od_q_slot(o, 0);
    if (served && q0 >= 0) m2_0 = od_q_m2(o, rec, q0, tq);
  }
  const double v0 = sqrt(m2_0);
  if constexpr (TR) { if (v0 != -1.0) pf_trace(tr, 4); }
  // rows 1.. (a history slot holds every node)
  double vsel = v0;
  const double* srow = rows_lds ? od_rows_put<M>(sh, a.n_out, rv) : nullptr;
  const double vfm = sqrt(fma(vf.y, vf.y, vf.x * vf.x));
  pf_rows_out<M>(t, rows_lds, srow, a.n_out, ir, ii, [&](int ro, double v) {
    v = (served && ro == o.resp_v_row) ? vfm : v;
    const int qs = od_q_slot(o, ro);
    if (served && qs >= 0) v = sqrt(od_q_m2(o, rec, qs, tq));
    if (valid && b.v_out) b.v_out[(int64_t)ro * n + e] = (Sto)v;
    vsel = (ro == c.vv_row) ? v : vsel;
  });
  if constexpr (TR) { if (vsel != -1.0) pf_trace(tr, 5); }
  if (!valid) return;
  if (b.v_out) b.v_out[e] = (Sto)v0;
  if (b.iters) b.iters[e] = it;
  if (c.coordinated) {
    const double vv = pymax(pymax(0.0, c.vv_lo - vsel), vsel - c.vv_hi);
    if (b.vv) b.vv[e] = (Sto)vv;
    const double share = (vv * c.vv_penalty) / (double)c.n_agents;
#pragma unroll
    for (int ag = 0; ag < PGW_MAX_AGENTS; ++ag)
      if (ag < c.n_agents) b.reward[(int64_t)ag * n + e] = (Sto)(rw[ag] + (Sto)(-share));
  }
  if constexpr (TR) pf_trace(tr, 6);
}

template <int M, class Bufs, bool TR = false>
__global__ void __launch_bounds__(kBlock) k_coord_pf_od(CoordPFArgs c, PFArgs a, ODArgs o, pgw_pf_tables t,
                                                        int64_t n, Bufs b) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  __shared__ ODShared<M> sh;
  coord_pf_od_env<M, Bufs, TR, false>(c, a, o, t, n, b, e, e < n, sh);
}

// The node records' lookup of the fused C4 step (od_resp_lookup_v's fields).
struct ODVLook {
  const double* resp_v;
  double resp_x0, resp_inv_h;
  int32_t resp_nseg;
  int32_t timing_only;      // PGW_STEP_NOLOOKUP (A/B timing only): no lookup, no list -- results wrong
};

// ---- the snap solve of one env by a whole wave --------------------------------
// The one-launch C4 step (k_coord_step_od<.., true>) solves the rare envs the
// node records leave (P in a guard zone or a bracket, off the grid) itself,
// one env at a time with the lookup wave, instead of listing them for a second
// launch: any launch after the 100-MB agents step costs ~4.6 us here
// (profiles/r06/c4_step_boundary_experiments.txt), the step without one 23.1
// against 25.3 us (ab_nolist.txt).  The lane-per-env solve (od_solve) keeps 256
// envs' currents in 148 KB of LDS at 1 wave per SIMD; this form needs ~15 KB
// and few registers, so the step kernel keeps its occupancy.
//   lane i < m      element i: its voltage u_i, its current I'_i and row i of
//                   the matvec (W'' staged in LDS, s_w[c][k][i]);
//   lane r (r + 32) check row r from the previous (new) currents (s_rows).
// Every value is formed with od_solve's operations in its order -- the
// current law of current_od, the matvec column by column from k = 0 as
// pf_column (A += Wr I, B += Wi I', C += (Wr+Wi)(I+I')), the rows as
// od_rows_sparse, dsum / jsum summed in k order; only maxima and minima (order
// free, od_max propagating NaN) are reduced across lanes -- so the count, the
// currents and the node-0 voltage equal the lane-per-env solve's bit for bit
// (tests/test_gpu_pf_od.py::test_od_split_step_bit_identical, every env forced
// to the solve).
struct ODWaveArgs {
  double sr0[PGW_PF_MAX_M], si0[PGW_PF_MAX_M], fr[PGW_PF_MAX_M], fi[PGW_PF_MAX_M];   // PFArgs's
  double y0r[PGW_PF_MAX_M], y0i[PGW_PF_MAX_M], esc[PGW_PF_MAX_M];                    // ODArgs's
  double lo2, mn2, mx2;                            // uniform bands (PFSolver<M, true, ..>)
  double tol, gamma, eps, gmax, gsrc;              // od_decide's
  const double* block;                             // the resident block (pgw_pf_tables.block)
  const double* start;                             // pgw_pf_od.start: u_1 and I'(u_0) affine in P, Q
  const double* rows_V0;
  const double* rows_G;
  int32_t m, min_iter, n_rep, n_rows, max_iter, node_mask;
};
constexpr int kWaveRowStride = 2 + 2 * PGW_PF_MAX_M + 1;   // odd: 32 rows on distinct banks
struct ODWaveShared {
  double w[3][PGW_PF_MAX_M][PGW_PF_MAX_M];         // [c][k][i] = part c of W''_ik
  double rows[kOdRows * kWaveRowStride];           // V0 re, im, G re (k), G im (k) per check row
  double el[9][PGW_PF_MAX_M];                      // per element: sr0 si0 fr fi y0r y0i esc u0re u0sum
  double st[12 * PGW_PF_MAX_M];                    // pgw_pf_od.start
};

__device__ __forceinline__ double wave_bcast(double x, int k) {   // lane k's value (k uniform)
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)(unsigned)(b & 0xffffffffll), k);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double wave_uni(double x) {     // a wave-uniform value, made scalar
  return wave_bcast(x, 0);
}
// (the partner lane's address from an opaque lane id: formed at use, not
// hoisted into registers held through the solve)
__device__ __forceinline__ double wave_xor(double x, int d) {
  int l = threadIdx.x & 63;
  asm volatile("" : "+v"(l));
  return __shfl(x, l ^ d);
}
// x from the lane CTRL names within its 16-lane row (DPP row_ror: no lane is
// without a source, so idempotent reductions need no identity)
template <int CTRL>
__device__ __forceinline__ double row_dpp(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
constexpr int kRowRor1 = 0x121, kRowRor2 = 0x122, kRowRor4 = 0x124, kRowRor8 = 0x128;
__device__ __forceinline__ double wave_max(double x) {     // od_max over the wave (uniform result)
  x = od_max(x, row_dpp<kRowRor1>(x));
  x = od_max(x, row_dpp<kRowRor2>(x));
  x = od_max(x, row_dpp<kRowRor4>(x));
  x = od_max(x, row_dpp<kRowRor8>(x));
  double r = wave_bcast(x, 0);
#pragma unroll 1
  for (int l = 16; l < 64; l += 16) r = od_max(r, wave_bcast(x, l));
  return r;
}
__device__ __forceinline__ double wave_min(double x) {
  x = fmin(x, row_dpp<kRowRor1>(x));
  x = fmin(x, row_dpp<kRowRor2>(x));
  x = fmin(x, row_dpp<kRowRor4>(x));
  x = fmin(x, row_dpp<kRowRor8>(x));
  double r = wave_bcast(x, 0);
#pragma unroll 1
  for (int l = 16; l < 64; l += 16) r = fmin(r, wave_bcast(x, l));
  return r;
}

// W'' and the check rows into the wave's LDS (the calling wave only).
__device__ __forceinline__ void od_wave_stage(const ODWaveArgs& z_, ODWaveShared& sh_) {
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));                   // (opaque: see od_wave_solve)
  const ODWaveArgs& z = z_;                        // (kernarg: scalar loads)
  ODWaveShared& sh = sh_;
  const int M = z.m, T = M * (M + 1) / 2;
  // every load of a batch in flight before its LDS stores (a load-store loop
  // waited one L2 round trip per entry: ~20 us per staged solve); the
  // addresses are clamped in bounds and the values selected after the load
  constexpr int kWq = 3 * PGW_PF_MAX_M * PGW_PF_MAX_M / 64;
  {
    double v[kWq];
#pragma unroll
    for (int q = 0; q < kWq; ++q) {
      const int x = lane + 64 * q;
      const int c = x / (PGW_PF_MAX_M * PGW_PF_MAX_M), k = (x / PGW_PF_MAX_M) % PGW_PF_MAX_M,
                i = x % PGW_PF_MAX_M;
      const int ic = min(i, M - 1), kc = min(k, M - 1);
      const int a = min(ic, kc), b = max(ic, kc);
      const double t = z.block[c * T + a * M - a * (a - 1) / 2 + (b - a)];
      v[q] = (i < M && k < M) ? t : 0.0;
    }
#pragma unroll
    for (int q = 0; q < kWq; ++q) (&sh.w[0][0][0])[lane + 64 * q] = v[q];
  }
  {
    // the per-element constants (kernarg, L2) and the start table, once per
    // wave instead of once per solve
    const int k = lane & 15, kc = min(k, M - 1);
    double v[12];
    v[0] = z.sr0[k];
    v[1] = z.si0[k];
    v[2] = z.fr[k];
    v[3] = z.fi[k];
    v[4] = z.y0r[k];
    v[5] = z.y0i[k];
    v[6] = z.esc[k];
    v[7] = z.block[3 * T + kc];
    v[8] = z.block[3 * T + 2 * M + kc];
#pragma unroll
    for (int q = 0; q < 3; ++q) v[9 + q] = z.start[min(lane + 64 * q, 12 * M - 1)];
    if (lane < PGW_PF_MAX_M) {
#pragma unroll
      for (int j = 0; j < 9; ++j) sh.el[j][lane] = v[j];
    }
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (lane + 64 * q < 12 * M) sh.st[lane + 64 * q] = v[9 + q];
  }
  const int S = 2 + 2 * M, nr = max(z.n_rows, 1);
  constexpr int kRq = 9;                             // entries per lane per batch
  for (int x0 = 0; x0 < z.n_rows * S; x0 += 64 * kRq) {   // (uniform: two batches at most)
    double v[kRq];
#pragma unroll
    for (int q = 0; q < kRq; ++q) {
      const int x = x0 + lane + 64 * q;
      const int r = min(x / S, nr - 1), j = x - (x / S) * S;
      v[q] = j < 2 ? z.rows_V0[2 * r + j]
                   : z.rows_G[2 * M * r + (j < 2 + M ? 2 * (j - 2) : 2 * (j - 2 - M) + 1)];
    }
#pragma unroll
    for (int q = 0; q < kRq; ++q) {
      const int x = x0 + lane + 64 * q;
      if (x < z.n_rows * S) sh.rows[(x / S) * kWaveRowStride + (x - (x / S) * S)] = v[q];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Rows [r0, r1) of the exact test (lane r: previous magnitude, lane r + 32:
// new), folded into (err, amin) of lanes < 32 (wave-reduced by the caller).
__device__ __forceinline__ void od_wave_rows(const ODWaveShared& sh, int M, int r0, int r1, double pjr,
                                             double pji, double cjr, double cji, double& err, double& amin) {
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));                   // (opaque: addresses formed here)
  const bool newer = lane >= 32;
  const int r = min(r0 + (lane & 31), max(r1 - 1, 0));
  const bool on = r0 + (lane & 31) < r1;
  const double* R = sh.rows + r * kWaveRowStride;
  double vr = R[0], vi = R[1];
#pragma unroll
  for (int k = 0; k < PGW_PF_MAX_M; ++k) {           // (uniform) od_rows_sparse's order
    if (k >= M) break;
    const double gr = R[2 + k], gi = R[2 + M + k];
    const double pr = wave_bcast(pjr, k), pi = wave_bcast(pji, k);
    const double cr = wave_bcast(cjr, k), ci = wave_bcast(cji, k);
    const double jx = newer ? cr : pr, jy = newer ? ci : pi;
    vr = fma(gr, jx, vr);
    vi = fma(gr, jy, vi);
    vr = fma(-gi, jy, vr);
    vi = fma(gi, jx, vi);
  }
  const double mg = od_mag(fma(vi, vi, vr * vr));
  const double mn = wave_xor(mg, 32);                // lanes < 32: the new magnitude
  const bool prev_lane = on && !newer;
  err = od_max(err, prev_lane ? fabs(mn - mg) : 0.0);
  amin = fmin(amin, prev_lane ? mg : __builtin_huge_val());
}

// The snap solve of the env with controllable powers (pc, qc) (uniform), by
// the whole wave (full EXEC); sh staged.  Returns the count (negative when
// stopped by max_iter) and leaves node 0's voltage (pf_node0's operations) in
// (v0r, v0i) of every lane.
__device__ int od_wave_solve(const ODWaveArgs& z_, const ODWaveShared& sh_, double pc, double qc, double& v0r,
                             double& v0i) {
  // (an opaque lane id: the solve's per-lane addresses are formed here, not
  // hoisted where they would hold registers through the agents' step; z stays
  // a kernarg reference -- laundering it made every z.* a per-iteration flat
  // load; the k loops have compile-time trip counts because readlane is
  // convergent and a runtime-count loop around it is not unrolled)
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));
  const ODWaveArgs& z = z_;                        // (kernarg: scalar loads)
  const ODWaveShared& sh = sh_;
  const int M = z.m, T = M * (M + 1) / 2;
  const int i = min(lane, M - 1);
  // (the per-element constants and the start table staged in LDS)
  const double sr0 = sh.el[0][i], si0 = sh.el[1][i], fr = sh.el[2][i], fi = sh.el[3][i];
  const double y0r = sh.el[4][i], y0i = sh.el[5][i], esc = sh.el[6][i];
  const bool node = lane < M && ((z.node_mask >> i) & 1);
  const double s_r = fma(fr, pc, sr0), s_i = fma(fi, qc, si0);   // pf_power's
  const double* st = sh.st;
  const double u0re = sh.el[7][i], u0sum = sh.el[8][i];
  // u_1 and the table currents I'(u_0) (od_solve's affine / currents_1)
  double ur = fma(qc, st[2 * (2 * M + i)], fma(pc, st[2 * (M + i)], st[2 * i]));
  double ui = fma(qc, st[2 * (2 * M + i) + 1], fma(pc, st[2 * (M + i) + 1], st[2 * i + 1]));
  const int c1 = 3 * M + i;
  double pjr = fma(qc, st[2 * (2 * M + c1)], fma(pc, st[2 * (M + c1)], st[2 * c1]));
  double pji = fma(qc, st[2 * (2 * M + c1) + 1], fma(pc, st[2 * (M + c1) + 1], st[2 * c1 + 1]));
  const double tol_lo = z.tol * (1.0 + 0x1p-30);
  const bool bounded = z.n_rep < z.n_rows;
  int it = 1, my_it = 1;
  bool conv_ok = false, done = z.max_iter <= 1;
  while (!done) {                                    // (uniform)
    ++it;
    // element i's current from u_{it-1} (current_od's operations)
    const double m2 = fma(ui, ui, ur * ur);
    double mc = fmin(fmax(m2, z.mn2), z.mx2);
    mc = (m2 <= z.lo2) ? 1.0 : mc;
    const double g = fast_rcp(mc);
    const double cr = fma(s_r, g, -y0r), ci = fma(s_i, g, -y0i);
    const double cjr = fma(cr, ur, -(ci * ui)), cji = fma(cr, ui, ci * ur);
    const double cjs = cjr + cji;
    // row i of the matvec, column by column (pf_acc_init, pf_column)
    double A = u0re, Bs = 0.0, C = u0sum;
    int ie = i;
    asm volatile("" : "+v"(ie));                     // (opaque: see od_wave_rows)
    const double* wk = &sh.w[0][0][0] + ie;
#pragma unroll
    for (int k = 0; k < PGW_PF_MAX_M; ++k) {         // (compile-time trip count, uniform guard)
      if (k < M) {
        A = fma(wk[k * PGW_PF_MAX_M], wave_bcast(cjr, k), A);
        Bs = fma(wk[(PGW_PF_MAX_M + k) * PGW_PF_MAX_M], wave_bcast(cji, k), Bs);
        C = fma(wk[(2 * PGW_PF_MAX_M + k) * PGW_PF_MAX_M], wave_bcast(cjs, k), C);
      }
    }
    const double nr = A - Bs, ni = (C - A) - Bs;
    // the square-root-free lower bound over the element nodes
    bool hit = false;
    double err = 0.0, amin = __builtin_huge_val();
    {
      const double e2 = esc * esc;
      const double a2 = fma(ni, ni, nr * nr) * e2, b2 = fma(ui, ui, ur * ur) * e2;
      hit = node && fabs(a2 - b2) > tol_lo * fma(0.5, a2 + b2, 1.0);
    }
    const bool need = it >= z.min_iter && __ballot(hit) == 0ull;   // (uniform)
    if (need) {
      const double mo = od_mag(fma(ui, ui, ur * ur)) * esc;
      const double mn = od_mag(fma(ni, ni, nr * nr)) * esc;
      err = node ? fabs(mn - mo) : 0.0;
      amin = node ? mo : __builtin_huge_val();
    }
    ur = nr;
    ui = ni;
    int d = 0;
    if (need) {
      double dsum = 0.0, jsum = 0.0;
#pragma unroll
      for (int k = 0; k < PGW_PF_MAX_M; ++k) {       // (uniform) in k order
        if (k >= M) break;
        const double cx = wave_bcast(cjr, k), cy = wave_bcast(cji, k);
        const double px = wave_bcast(pjr, k), py = wave_bcast(pji, k);
        dsum += fabs(cx - px) + fabs(cy - py);
        jsum += fabs(px) + fabs(py);
      }
      dsum = wave_uni(fma(0x1p-40, jsum + dsum, dsum));
      jsum = wave_uni(fma(0x1p-40, jsum, jsum));
      for (int r0 = 0; r0 < z.n_rep; r0 += 32)
        od_wave_rows(sh, M, r0, min(r0 + 32, z.n_rep), pjr, pji, cjr, cji, err, amin);
      double lo = wave_uni(wave_max(err)), am = wave_uni(wave_min(amin));
      d = __builtin_amdgcn_readfirstlane(od_decide(z, !bounded, it, lo, am, dsum, jsum));
      if (d < 0) {                                   // (uniform) the bounded rows decide
        for (int r0 = z.n_rep; r0 < z.n_rows; r0 += 32)
          od_wave_rows(sh, M, r0, min(r0 + 32, z.n_rows), pjr, pji, cjr, cji, err, amin);
        lo = wave_uni(wave_max(err));
        am = wave_uni(wave_min(amin));
        d = __builtin_amdgcn_readfirstlane(od_decide(z, true, it, lo, am, dsum, jsum));
      }
    }
    pjr = cjr;                                       // this iteration's currents: the next one's
    pji = cji;                                       // previous, and the outputs' when it stops
    my_it = it;
    conv_ok = d > 0;
    done = d > 0 || it >= z.max_iter;
  }
  // node 0 from the accepted currents (pf_node0's operations)
  const double* B = z.block + 3 * T + 6 * M;         // g0re[M], g0im[M], v0re, v0im
  double vr = B[2 * M], vi = B[2 * M + 1];
#pragma unroll 4
  for (int k = 0; k < M; ++k) {                      // (uniform)
    const double gr = B[k], gi = B[M + k];
    const double jr = wave_bcast(pjr, k), ji = wave_bcast(pji, k);
    vr = fma(gr, jr, vr);
    vi = fma(gr, ji, vi);
    vr = fma(-gi, ji, vr);
    vi = fma(gi, jr, vi);
  }
  v0r = vr;
  v0i = vi;
  return conv_ok ? my_it : -my_it;
}

// Fused C4 step, OpenDSS rule with the hour's node records (pgw_pf_od.resp_v,
// output row 0 the coordinated bus, no other row): the agents AND the power
// flow's table lookup in one launch.  A block is n_agents waves over 64 envs;
// wave a runs agent a's step (std_agent_compute, k_coord_agents_std's
// operations and stores) and leaves its real power in LDS; after the block
// barrier wave 0 sums the bus load in agent order (k_coord_pf_od's prologue),
// looks the env up in the node records and, where the table serves it, writes
// V675.3, the violation and the iteration count and leaves the reward share in
// LDS; every wave then stores its agent's final reward (raw + (-share), as
// k_coord_pf_od's epilogue).  Envs the table does not serve keep their raw
// rewards and are appended to b.od_list (count b.od_count[parity]) for
// k_coord_pf_od_list, launched next.  Block 0 zeroes the other parity's count
// (the next step's list).  Bit-identical to k_coord_agents_std + k_coord_pf_od.
// WT: every store write-through (st_wt), so the step leaves no dirty L2 lines
// for the next launch's boundary to write back.
// INL (the default one-launch step): the lookup wave solves the envs the table
// leaves itself (od_wave_solve), one at a time, and nothing is listed -- the
// step is this launch alone.  (7 waves per SIMD: 71 VGPRs, 5 blocks per CU;
// at 6 the kernel ran 0.3 us slower, profiles/r06/ab_one_launch_step.txt.)
// (the step's parameters and the wave solve's constants: one first argument,
// read in place from the kernarg segment)
struct StepOdArgs {
  pgw_coord_params p;
  ODWaveArgs z;
};
template <bool WT, bool INL>
__global__ void __launch_bounds__(64 * PGW_MAX_AGENTS) __attribute__((amdgpu_waves_per_eu(7))) k_coord_step_od(StepOdArgs A_, pgw_coord_step_info s,
                                                                       int64_t n, pgw_coord_buffers b, double pv_ob,
                                                                       StdDerived dv, CoordPFArgs c, ODVLook o) {
  auto put = [](auto* q, auto v) {
    if constexpr (WT) st_wt(q, v);
    else *q = v;
  };
  const StepOdArgs& A = PGW_KERNARG0(StepOdArgs);               // (no private copy)
  const pgw_coord_params& p = A.p;
  const ODWaveArgs& z = A.z;
  const int a = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * 64 + lane;
  const bool valid = e < n;
  __shared__ double s_pow[PGW_MAX_AGENTS][64];
  __shared__ double s_share[64];
  __shared__ int s_served[64];
  if (blockIdx.x == 0 && threadIdx.x == 0) b.od_count[(b.od_parity & 1) ^ 1] = 0;
  double rw = 0.0;
  if (valid) {
    StdAgentIn in[1];
    const double* ap = b.action.ptr + a * b.act_stride_agent + e * b.action.s_env;
#pragma unroll
    for (int j = 0; j < 8; ++j) in[0].av[j] = ld_act(ap + j * b.action.s_dim);
    double* xp = b.x + (int64_t)a * 5 * n + e;
#pragma unroll
    for (int z = 0; z < 5; ++z) in[0].xs[z] = xp[z * n];
    double* socp = b.soc + (int64_t)a * n + e;
    in[0].soc = *socp;
    double* op = b.obs.ptr + a * b.obs_stride_agent + e * b.obs.s_env;
    std_agent_compute<1>(p, dv, s, pv_ob, in, [&](int slot, const double (&v)[1]) {
      if (slot < kSlotSoc) put(xp + slot * n, v[0]);
      else if (slot == kSlotSoc) put(socp, v[0]);
      else if (slot < kSlotPower) {
        if constexpr (WT) st_wt(op + (slot - kSlotObs) * b.obs.s_dim, v[0]);
        else st_obs(op + (slot - kSlotObs) * b.obs.s_dim, v[0]);
      } else if (slot == kSlotPower) {
        put(b.agent_power + (int64_t)a * n + e, v[0]);
        s_pow[a][lane] = v[0];
      } else {
        rw = v[0];
      }
    });
  }
  __syncthreads();
  if (a == 0) {
    // the bus load of controllable slot 0 in agent order (k_coord_pf_od: 0 + p0 + p1 ...)
    double pc = 0.0;
#pragma unroll
    for (int ag = 0; ag < PGW_MAX_AGENTS; ++ag) {
      const int slot = ag < c.n_agents ? c.agent_ctrl[ag] : -1;
      const double rp = (valid && ag < c.n_agents) ? s_pow[ag][lane] * 1.0 : 0.0;
      pc = (slot == 0) ? pc + rp : pc;
    }
    double2 vf = make_double2(0.0, 0.0);
    int it = 0;
    // (a local copy: a reference to the by-value kernel argument would put it
    // in a private-memory frame)
    const ODVLook ol = {o.resp_v, o.resp_x0, o.resp_inv_h, o.resp_nseg, 0};
    bool served = valid && !o.timing_only && od_resp_lookup_v(ol, pc, 0.0, vf, it);
    if constexpr (INL) {
      // the envs the table left: the wave's snap solve, one env at a time
      // (the usual wave has none); their node-0 voltage then takes the served
      // path's place (the same operations as k_coord_pf_od's epilogue)
      __shared__ ODWaveShared s_solve;
      uint64_t left = __ballot(valid && !served && !o.timing_only);
      if (left) {                                    // (uniform) counted as the list form counts them
        if (lane == 0) atomicAdd(b.od_count + (b.od_parity & 1), __popcll(left));
        od_wave_stage(z, s_solve);
      }
      while (left) {                                 // (uniform)
        const int L = __builtin_ctzll(left);
        left &= left - 1;
        double v0r, v0i;
        const int its = od_wave_solve(z, s_solve, wave_bcast(pc, L), 0.0, v0r, v0i);
        if (lane == L) {
          vf = make_double2(v0r, v0i);
          it = its;
          served = true;
        }
      }
    }
    double share = 0.0;
    if (served) {
      const double v0 = sqrt(fma(vf.y, vf.y, vf.x * vf.x));
      if (b.v_out) put(b.v_out + e, v0);
      if (b.iters) put(b.iters + e, (int32_t)it);
      if (c.coordinated) {
        const double vv = pymax(pymax(0.0, c.vv_lo - v0), v0 - c.vv_hi);
        if (b.vv) put(b.vv + e, vv);
        share = (vv * c.vv_penalty) / (double)c.n_agents;
      }
    }
    // the envs left to the solve: one list slot each, one atomic per wave
    // (INL: none -- every valid env was served or solved above)
    const bool need = !INL && valid && !served && !o.timing_only;
    const uint64_t m = __ballot(need);
    if (m) {
      const int first = __builtin_ctzll(m);
      int base = 0;
      if (lane == first) base = atomicAdd(b.od_count + (b.od_parity & 1), __popcll(m));
      base = __shfl(base, first);
      if (need) b.od_list[base + __popcll(m & ((1ull << lane) - 1ull))] = (int32_t)e;
    }
    s_share[lane] = share;
    s_served[lane] = served ? 1 : 0;
  }
  __syncthreads();
  if (!valid) return;
  const bool fin = c.coordinated && s_served[lane];
  put(b.reward + (int64_t)a * n + e, fin ? rw + (-s_share[lane]) : rw);
}

// The snap solve of the envs k_coord_step_od appended to its list (the table
// did not serve them: P in a bracket or a guard zone, off the grid, an unfit
// piece), grid-stride over the list with a small fixed grid: the list's count
// is read once, so with nothing to solve (the usual step) every block exits
// after one load.  Outputs as k_coord_pf_od's for these envs.
template <int M, bool LOOP>
__global__ void __launch_bounds__(kBlock) k_coord_pf_od_list(CoordPFArgs c, PFArgs a, ODArgs o, pgw_pf_tables t,
                                                             int64_t n, pgw_coord_buffers b) {
  const int32_t cnt = b.od_count[b.od_parity & 1];     // (uniform)
  if ((int64_t)blockIdx.x * kBlock >= cnt) return;     // (block-uniform)
  __shared__ ODShared<M> sh;
  if constexpr (LOOP) {
    for (int64_t base = (int64_t)blockIdx.x * kBlock; base < cnt; base += (int64_t)gridDim.x * kBlock) {
      const int64_t i = base + threadIdx.x;
      const bool valid = i < cnt;
      const int64_t e = valid ? (int64_t)b.od_list[i] : 0;
      coord_pf_od_env<M, pgw_coord_buffers, false, true>(c, a, o, t, n, b, e, valid, sh);
      __syncthreads();                                 // (the next pass re-stages sh)
    }
  } else {                                             // one block per 256 list slots
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const bool valid = i < cnt;
    const int64_t e = valid ? (int64_t)b.od_list[i] : 0;
    coord_pf_od_env<M, pgw_coord_buffers, false, true>(c, a, o, t, n, b, e, valid, sh);
  }
}

// pgw_pf_solve, OpenDSS rule: k_pf_solve's prologue (the env's controllable
// powers) and outputs (every output row from the accepted iteration's currents
// -- staged in the solve's LDS after it, od_rows_put --, extrema, element
// voltages), the response table / snap solve in between.
template <int M, class IO = double>
__global__ void __launch_bounds__(kBlock) k_pf_solve_od(PFArgs a, ODArgs o, pgw_pf_tables t, int64_t n,
                                                        const IO* __restrict__ ctrl_p,
                                                        const IO* __restrict__ ctrl_q,
                                                        IO* __restrict__ v_out,
                                                        int32_t* __restrict__ iters) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool valid = e < n;
  __shared__ ODShared<M> sh;
  ODStage<M> stg;
  // the table gives currents, not element voltages: U_out asks for the solve
  const bool table = o.resp != nullptr && t.U_out == nullptr;
  const bool rows_lds = od_rows_lds<M>(a.n_out);     // (uniform)
  // extrema only with row records covering every candidate row (and row 0):
  // a block the table serves entirely reads the row records' headers and
  // quartics alone -- no currents, no node-0 or row DPP groups, no row staging
  const bool qfast = table && v_out == nullptr && o.resp_q && rows_lds && o.resp_rows != 0 &&
                     (od_q_slot(o, 0) >= 0 || o.resp_v_row == 0);        // (uniform)
  double rv[kOdRowQ];
  PFSolver<M, true, false> S;
  // the solve's operands (the block, the output rows) go out first -- in
  // flight with the env's powers -- except in qfast launches, where a block
  // the table serves entirely never uses them: there the env's powers go out
  // alone and the operands follow only for a block with an env left over
  if (!qfast) {                                      // (uniform)
    if (!table) od_stage_load<M>(o, o.start, stg);
    if (rows_lds) od_rows_issue<M>(t, a.n_out, rv);
    S.load(a, t.block);
  }
  double cp[PGW_PF_MAX_CTRL], cq[PGW_PF_MAX_CTRL];
#pragma unroll
  for (int c = 0; c < PGW_PF_MAX_CTRL; ++c) {
    cp[c] = (valid && c < a.n_ctrl && ctrl_p) ? (double)ctrl_p[(int64_t)c * n + e] : 0.0;
    cq[c] = (valid && c < a.n_ctrl && ctrl_q) ? (double)ctrl_q[(int64_t)c * n + e] : 0.0;
  }
  S.powers(a, cp, cq, 1.0);
  double ir[M], ii[M], v0r, v0i;
#pragma unroll
  for (int k = 0; k < M; ++k) ir[k] = ii[k] = 0.0;
  int it = 0;
  double2 vf = make_double2(0.0, 0.0);
  int rec = 0;
  double tq = 0.0;
  uint64_t qm = ~0ull;                               // the record's candidate slots (od_q_cand)
  bool served, blk_fast = false;
  if (qfast) {
    served = valid && od_q_find(o, S.pc, S.qc, it, rec, tq, qm);
    if (served && o.resp_v) {
      const double2* vr = reinterpret_cast<const double2*>(o.resp_v) + (int64_t)rec * (PGW_OD_VREC / 2);
      vf = od_rec_j(vr[3], vr[4], vr[5], tq);
    }
    blk_fast = !__syncthreads_or(valid && !served);   // (block-uniform)
    if (!blk_fast) {                                 // the operands the solve and the rows need
      od_rows_issue<M>(t, a.n_out, rv);
      S.load(a, t.block);
      if (served) od_resp_at<M>(o, rec, tq, ir, ii, vf);
    } else {
#pragma unroll
      for (int q = 0; q < kOdRowQ; ++q) rv[q] = 0.0;   // (never read)
    }
  } else {
    served = valid && table && od_resp_lookup<M>(o, S.pc, S.qc, ir, ii, it, vf, rec, tq);
    if (served && o.resp_q) qm = od_q_cand(o.resp_q[(int64_t)rec * o.resp_q_stride + 5]);
  }
  const bool need = valid && !served;
  od_fallback<M>(S, o, o.start, stg, table, sh, need, ir, ii, it);
  v0r = v0i = 0.0;
  if (!blk_fast) pf_node0<M>(v0r, v0i, S.w, ir, ii);
  if (served && o.resp_v_row == 0) {                 // the node record's row
    v0r = vf.x;
    v0i = vf.y;
  }
  double m2_0 = fma(v0i, v0i, v0r * v0r);
  if (o.resp_q) {                                    // (uniform) the row records' row 0
    const int q0 = od_q_slot(o, 0);
    if (served && q0 >= 0) m2_0 = od_q_m2(o, rec, q0, tq);
  }
  const double v0 = sqrt(m2_0);
  const double vf2 = fma(vf.y, vf.y, vf.x * vf.x);
  if (valid && t.U_out) {
#pragma unroll
    for (int k = 0; k < M; ++k) {
      t.U_out[2 * (e * M + k)] = S.ur[k];
      t.U_out[2 * (e * M + k) + 1] = S.ui[k];
    }
  }
  double vmn = v0, vmx = v0;      // Python min()/max() over the rows in order
  const double* srow = (rows_lds && !blk_fast) ? od_rows_put<M>(sh, a.n_out, rv) : nullptr;
  if (v_out || !rows_lds) {
    const double vfm = sqrt(vf2);
    pf_rows_out<M>(t, rows_lds, srow, a.n_out, ir, ii, [&](int ro, double v) {
      v = (served && ro == o.resp_v_row) ? vfm : v;
      const int qs = od_q_slot(o, ro);
      if (served && qs >= 0) v = sqrt(od_q_m2(o, rec, qs, tq));
      if (valid && v_out) v_out[(int64_t)ro * n + e] = (IO)v;
      vmn = (v < vmn) ? v : vmn;
      vmx = (v > vmx) ? v : vmx;
    });
  } else {
    // extrema only: min / max of |V|^2 over the rows, one sqrt each at the end
    // (as k_pf_solve: sqrt is monotone and correctly rounded)
    double mn2 = m2_0, mx2 = mn2;
    auto ext = [&](int ro, double m2) {
      m2 = (served && ro == o.resp_v_row) ? vf2 : m2;
      const int qs = od_q_slot(o, ro);
      if (served && qs >= 0) {
        if (!((qm >> qs) & 1ull)) return;            // not this record's candidate: never its extremum
        m2 = od_q_m2(o, rec, qs, tq);
      }
      mn2 = (m2 < mn2) ? m2 : mn2;
      mx2 = (m2 > mx2) ? m2 : mx2;
    };
    const uint64_t cand = o.resp_rows | (o.resp_v_row > 0 ? 1ull << o.resp_v_row : 0ull);
    if (blk_fast) {
      // the candidate rows in order from the row records (and the node record),
      // the values the masked DPP path below gives them
      uint64_t m = a.n_out < 64 ? cand & ((1ull << a.n_out) - 1ull) & ~1ull : cand & ~1ull;
      while (m) {                                    // (uniform)
        const int ro = __builtin_ctzll(m);
        m &= m - 1;
        ext(ro, 0.0);
      }
    } else if (rows_lds && o.resp_rows != 0 && __ballot(valid && !served) == 0ull) {
      // only the rows that can hold a served env's extremum (pgw_pf_od.resp_rows),
      // unless an env of this wave was solved in full
      pf_rows_mask2<M>(srow, a.n_out, cand, ir, ii, ext);
    } else {
      pf_rows_out<M, false>(t, rows_lds, srow, a.n_out, ir, ii, ext);
    }
    vmn = sqrt(mn2);
    vmx = sqrt(mx2);
  }
  if (!valid) return;
  if (a.n_out > 0) {
    if (v_out) v_out[e] = (IO)v0;
    if (t.v_min_out) t.v_min_out[e] = vmn;
    if (t.v_max_out) t.v_max_out[e] = vmx;
  }
  if (iters) iters[e] = it;
}

// Response-table builder (pgw_pf_od_probe): the snap solve at lane e's kW P[e]
// (Q = 0) in hour e / lanes_per_hour -- that hour's PFArgs (base loads) and
// first-iteration table -- with the signature of its pieces.
template <int M>
__global__ void __launch_bounds__(kBlock) k_pf_od_probe(const PFArgs* __restrict__ args_h, ODArgs o,
                                                        pgw_pf_tables t, const double* __restrict__ start_h,
                                                        int32_t lanes_per_hour, int64_t n,
                                                        const double* __restrict__ P,
                                                        double2* __restrict__ J_out, uint64_t* __restrict__ sig_out,
                                                        int32_t* __restrict__ it_out) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool valid = e < n;
  const int hour = (int)(((int64_t)blockIdx.x * kBlock) / lanes_per_hour);   // (block-uniform)
  const PFArgs& a = args_h[hour];
  const double* start = start_h + (int64_t)hour * 12 * M;
  __shared__ ODShared<M> sh;
  ODStage<M> stg;
  od_stage_load<M>(o, start, stg);
  PFSolver<M, true, false> S;
  S.load(a, t.block);
  double cp[PGW_PF_MAX_CTRL], cq[PGW_PF_MAX_CTRL];
#pragma unroll
  for (int c = 0; c < PGW_PF_MAX_CTRL; ++c) {
    cp[c] = (valid && c == 0) ? P[e] : 0.0;
    cq[c] = 0.0;
  }
  S.powers(a, cp, cq, 1.0);
  od_stage_store<M>(o, stg, sh);
  __syncthreads();
  uint64_t sig = kFnvBasis;
  const int it = od_solve<M, true>(S, o, stg, valid, sh, &sig);
  double ir[M], ii[M];
  od_load_J<M>(sh, it, ir, ii);
  if (!valid) return;
#pragma unroll
  for (int k = 0; k < M; ++k) J_out[e * M + k] = make_double2(ir[k], ii[k]);
  sig_out[e] = sig;
  it_out[e] = it;
}

// Pieces -> records (pgw_pf_od_resp_fit), one thread per piece.
__global__ void __launch_bounds__(kBlock) k_pf_od_resp_fit(int32_t m, int64_t np, const double2* __restrict__ J,
                                                           const int32_t* __restrict__ idx3,
                                                           const double* __restrict__ meta,
                                                           const int32_t* __restrict__ inext,
                                                           const int32_t* __restrict__ rec, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= np) return;
  double* o = out + (int64_t)rec[i] * PGW_OD_REC(m);
  for (int q = 0; q < 4; ++q) o[q] = meta[4 * i + q];
  const unsigned long long packed =
      (unsigned long long)(uint32_t)inext[2 * i] | ((unsigned long long)(uint32_t)inext[2 * i + 1] << 32);
  o[4] = __longlong_as_double((long long)packed);
  o[5] = 0.0;
  const double2* ja = J + (int64_t)idx3[3 * i] * m;
  const double2* jm = J + (int64_t)idx3[3 * i + 1] * m;
  const double2* jb = J + (int64_t)idx3[3 * i + 2] * m;
  double* c = o + PGW_OD_REC_HEAD;
  for (int k = 0; k < m; ++k) {
    const double2 a = ja[k], md = jm[k], b = jb[k];
    c[2 * k] = md.x;
    c[2 * k + 1] = md.y;
    c[2 * m + 2 * k] = 0.5 * (b.x - a.x);
    c[2 * m + 2 * k + 1] = 0.5 * (b.y - a.y);
    c[4 * m + 2 * k] = 0.5 * (a.x + b.x) - md.x;
    c[4 * m + 2 * k + 1] = 0.5 * (a.y + b.y) - md.y;
  }
}

// Fit check (pgw_pf_od_resp_check), one thread per check point.
__global__ void __launch_bounds__(kBlock) k_pf_od_resp_check(int32_t m, int64_t n, const double* __restrict__ recs,
                                                             const int32_t* __restrict__ rec,
                                                             const double* __restrict__ P,
                                                             const double2* __restrict__ J,
                                                             const int32_t* __restrict__ iq,
                                                             double* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const double2* r = reinterpret_cast<const double2*>(recs + (int64_t)rec[i] * PGW_OD_REC(m));
  const double t = (P[i] - r[1].x) * r[1].y;
  const double2* jt = J + (int64_t)iq[i] * m;
  double num = 0.0, den = 0.0;
  for (int k = 0; k < m; ++k) {
    const double2 f = od_rec_j(r[3 + k], r[3 + m + k], r[3 + 2 * m + k], t);
    const double2 w = jt[k];
    num = fmax(num, hypot(f.x - w.x, f.y - w.y));
    den = fmax(den, hypot(w.x, w.y));
  }
  err[i] = den > 0.0 ? num / den : num;
}

// Stencil metadata of the predictor grid (one thread per segment): in a
// segment whose two ends share the band signature the switch sits at t* = 1/2
// (the nearest-point rule) and both sides use a 3-point stencil of that
// signature around the segment; in a segment where the signature changes, t*
// is where the first switching element's |u|^2 crosses its band limit (Newton
// on one side's quadratic, from the linear estimate) and each side takes the
// nearest 3 points of its own signature.  No matching stencil -> the plain one.
__global__ void __launch_bounds__(kBlock) k_pf_pred_meta(pgw_pf_params p, int32_t n_tables,
                                                         int32_t P, const double* __restrict__ U,
                                                         const int32_t* __restrict__ S,
                                                         pgw_pred_meta* __restrict__ meta) {
  const int64_t id = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t nseg = P - 1;
  if (id >= (int64_t)n_tables * nseg) return;
  const int tab = (int)(id / nseg), j = (int)(id - (int64_t)tab * nseg);
  const int32_t* Sg = S + (int64_t)tab * P;
  const double2* Ut = reinterpret_cast<const double2*>(U) + (int64_t)tab * P * p.m;
  auto same = [&](int a, int32_t sg) {
    return a >= 0 && a + 2 <= P - 1 && Sg[a] == sg && Sg[a + 1] == sg && Sg[a + 2] == sg;
  };
  const int plain_l = max(0, min(j - 1, P - 3)), plain_r = max(0, min(j, P - 3));
  pgw_pred_meta m;
  m.tstar = 0.5;
  m.left = plain_l;
  m.right = plain_r;
  const int32_t s0 = Sg[j], s1 = Sg[j + 1];
  if (s0 == s1) {
    const int cl[4] = {j - 1, j, j - 2, j + 1}, cr[4] = {j, j - 1, j + 1, j - 2};
    for (int q = 3; q >= 0; --q) {
      if (same(cl[q], s0)) m.left = cl[q];
      if (same(cr[q], s0)) m.right = cr[q];
    }
  } else {
    bool have_left = false;
    if (same(j - 2, s0)) { m.left = j - 2; have_left = true; }
    else if (same(j - 3, s0)) { m.left = j - 3; have_left = true; }
    if (same(j + 1, s1)) m.right = j + 1;
    else if (same(j + 2, s1)) m.right = j + 2;
    // the first element whose band differs between the two ends
    for (int k = 0; k < p.m; ++k) {
      const int b0 = (s0 >> (2 * k)) & 3, b1 = (s1 >> (2 * k)) & 3;
      if (b0 == b1) continue;
      const int lvl = min(b0, b1);   // boundary between band lvl and lvl + 1
      const double lim = lvl == 0 ? p.vlow[k] : lvl == 1 ? p.vmin[k] : p.vmax[k];
      const double thr = lim * lim;
      const double2 ua = Ut[(int64_t)j * p.m + k], ub = Ut[(int64_t)(j + 1) * p.m + k];
      const double m0 = ua.x * ua.x + ua.y * ua.y, m1 = ub.x * ub.x + ub.y * ub.y;
      double ts = (m1 != m0) ? fmin(fmax((thr - m0) / (m1 - m0), 0.0), 1.0) : 0.5;
      // refine: where the quadratic of one side (smooth up to the switch) crosses
      // the limit -- the linear estimate is off by a sliver of the segment, and
      // envs in that sliver would start from the other side's quadratic
      const int c = (have_left ? m.left : m.right) + 1;
      const double2 um = Ut[(int64_t)(c - 1) * p.m + k], u0 = Ut[(int64_t)c * p.m + k],
                    up = Ut[(int64_t)(c + 1) * p.m + k];
      const double d1r = 0.5 * (up.x - um.x), d1i = 0.5 * (up.y - um.y);
      const double d2r = 0.5 * (up.x - 2.0 * u0.x + um.x), d2i = 0.5 * (up.y - 2.0 * u0.y + um.y);
      for (int q = 0; q < 8; ++q) {
        const double tau = (double)(j - c) + ts;
        const double ur = u0.x + tau * (d1r + tau * d2r), ui = u0.y + tau * (d1i + tau * d2i);
        const double dr = d1r + 2.0 * tau * d2r, di = d1i + 2.0 * tau * d2i;
        const double f = ur * ur + ui * ui - thr, fp = 2.0 * (ur * dr + ui * di);
        if (fp == 0.0) break;
        ts = ts - f / fp;
      }
      m.tstar = fmin(fmax(ts, 0.0), 1.0);
      break;
    }
  }
  m.left += 1;      // stencil start -> record (centre) index
  m.right += 1;
  meta[id] = m;
}

// Predictor records (one thread per grid point): value fp64 + centred first and
// second differences fp32 (end points take their interior neighbour's).
template <int M>
__global__ void __launch_bounds__(kBlock) k_pf_pred_pack(int32_t n_tables, int32_t P,
                                                         const double* __restrict__ U,
                                                         double* __restrict__ rec) {
  const int64_t id = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (id >= (int64_t)n_tables * P) return;
  const int tab = (int)(id / P), j = (int)(id - (int64_t)tab * P);
  const int cj = min(max(j, 1), P - 2);
  const double2* Ut = reinterpret_cast<const double2*>(U) + (int64_t)tab * P * M;
  char* r = reinterpret_cast<char*>(rec) + id * (32 * M);
  double2* v = reinterpret_cast<double2*>(r);
  float2* d1 = reinterpret_cast<float2*>(r + 16 * M);
  float2* d2 = reinterpret_cast<float2*>(r + 24 * M);
#pragma unroll
  for (int k = 0; k < M; ++k) {
    const double2 um = Ut[(int64_t)(cj - 1) * M + k], u0 = Ut[(int64_t)cj * M + k],
                  up = Ut[(int64_t)(cj + 1) * M + k];
    v[k] = Ut[(int64_t)j * M + k];
    // differences about cj; a record at j != cj (grid ends) re-centres: with
    // s = j - cj, u_j + t d1/2 + t^2 d2/2 must equal the quadratic of cj at t + s
    const double s = (double)(j - cj);
    const double g1r = (up.x - um.x) + s * 2.0 * (up.x - 2.0 * u0.x + um.x);
    const double g1i = (up.y - um.y) + s * 2.0 * (up.y - 2.0 * u0.y + um.y);
    d1[k] = make_float2((float)g1r, (float)g1i);
    d2[k] = make_float2((float)(up.x - 2.0 * u0.x + um.x), (float)(up.y - 2.0 * u0.y + um.y));
  }
}

// Kernel instantiations: the element count is a template parameter so the
// matvec is fully unrolled with compile-time block offsets.
static int padded_m(int m) { return m <= 8 ? 8 : (m <= 14 ? 14 : 16); }

static bool uniform_band(const pgw_pf_params& p) {
  for (int k = 1; k < p.m; ++k)
    if (p.vlow[k] != p.vlow[0] || p.vmin[k] != p.vmin[0] || p.vmax[k] != p.vmax[0]) return false;
  return true;
}

static PFArgs make_pf_args(const pgw_pf_params& p, const pgw_pf_tables& t) {
  PFArgs a = {};
  for (int k = 0; k < PGW_PF_MAX_M; ++k) {
    const bool real = k < p.m;
    const double nph = real ? p.nph[k] : 1.0;
    const double sw = real ? (p.base_kw[k] * 1000.0) / nph : 0.0;
    const double sv = real ? (p.base_kvar[k] * 1000.0) / nph : 0.0;
    const int c = real ? p.elem_ctrl[k] : -1;
    a.sr0[k] = sw;
    a.si0[k] = -sv;
    a.fr[k] = (c == 0) ? 1000.0 / nph : 0.0;
    a.fi[k] = (c == 0) ? -1000.0 / nph : 0.0;
    a.kw[k] = real ? p.base_kw[k] : 0.0;
    a.kvar[k] = real ? p.base_kvar[k] : 0.0;
    a.nph[k] = nph;
    a.ctrl[k] = c;
  }
  a.lo2 = p.vlow[0] * p.vlow[0];
  a.mn2 = p.vmin[0] * p.vmin[0];
  a.mx2 = p.vmax[0] * p.vmax[0];
  a.tol2 = p.tol * p.tol;
  a.pred_x0 = p.pred_x0;
  a.pred_inv_h = p.pred_h != 0.0 ? 1.0 / p.pred_h : 0.0;
  a.pred_n = p.pred_n;
  a.use_pred = (t.U_pred != nullptr && p.n_ctrl == 1 && p.pred_n >= 3 && p.pred_h > 0.0) ? 1 : 0;
  a.max_iter = p.max_iter;
  a.n_ctrl = p.n_ctrl;
  a.n_out = p.n_out;
  return a;
}

template <int M, bool UB, bool GC, bool KEEP, class IO>
static int32_t launch_pf_solve(const PFArgs& a, const pgw_pf_tables& t, int64_t n, const IO* cp,
                               const IO* cq, IO* v_out, int32_t* iters, hipStream_t st) {
  launch_timed(PGW_T_PF_SOLVE, k_pf_solve<M, UB, GC, KEEP, IO>, dim3(grid_for(n)), dim3(kBlock), st, a, t, n,
               cp, cq, v_out, iters);
  return check_launch("k_pf_solve");
}

template <int M, bool UB, bool GC, bool KEEP, class Bufs>
static int32_t launch_coord_pf(const CoordPFArgs& c, const PFArgs& a, const pgw_pf_tables& t,
                               int64_t n, const Bufs& b, hipStream_t st) {
  launch_timed(PGW_T_COORD_PF, k_coord_pf<M, UB, GC, KEEP, Bufs>, dim3(grid_for(n)), dim3(kBlock), st, c, a,
               t, n, b);
  return check_launch("k_coord_pf");
}

// ThisPVEnv.step_reward (scenarios/heterogeneous.py:47-52) on [n]: Python's
// min(0, x) keeps 0 unless x < 0; (1000 viol)**2 as the square.
__global__ void __launch_bounds__(kBlock) k_band_penalty(int64_t n, const double* __restrict__ v,
                                                         double lo, double hi, double scale,
                                                         double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  const double x = v[e];
  const double l = x - lo, u = hi - x;
  const double viol = ((l < 0.0) ? l : 0.0) + ((u < 0.0) ? u : 0.0);
  const double y = scale * viol;
  out[e] = -(y * y);
}

// OpenDSS rule on the fast kernels (pgw_pf_tables.od): the C4 shape only.
static int32_t check_od(const pgw_pf_params& p, const pgw_pf_tables& t, const char* who) {
  const pgw_pf_od* d = t.od;
  PGW_REQUIRE(p.m == 14 && uniform_band(p) && p.n_ctrl <= 1 && !t.load_scale && !t.U_init,
              "%s: the OpenDSS fast path needs m = 14, one voltage band, <= 1 controllable slot and no "
              "load_scale / U_init (use pgw_pf_solve_general)", who);
  PGW_REQUIRE(d->n_rows >= 0 && d->n_rows <= PGW_PF_OD_MAX_ROWS && d->n_rep >= 0 && d->n_rep <= d->n_rows,
              "%s: od n_rep %d / n_rows %d (<= %d)", who, d->n_rep, d->n_rows, PGW_PF_OD_MAX_ROWS);
  PGW_REQUIRE(d->start && (d->n_rows == 0 || (d->rows_V0 && d->rows_G)), "%s: od start / rows missing", who);
  PGW_REQUIRE(d->min_iter >= 2 && p.max_iter >= 1 && d->tol >= 0.0, "%s: od min_iter / max_iter / tol", who);
  return PGW_OK;
}

// Instantiated variants: IEEE-13 (m = 14) with a uniform band, at most one
// controllable slot and no per-env load scale is the fast path (with one
// output row accumulated inside the loop, or the last currents kept for any
// number of rows); everything else runs the general variant (per-lane element
// powers) of its padded size.
#define PGW_PF_DISPATCH(p, t, fn, ...)                                     \
  do {                                                                     \
    const bool ub_ = uniform_band(p), gc_ = (p).n_ctrl > 1 || (t).load_scale; \
    switch ((p).m) {                                                       \
      case 8: return fn<8, false, true, true>(__VA_ARGS__);                \
      case 14:                                                             \
        if (ub_ && !gc_ && (p).n_out <= 1)                                 \
          return fn<14, true, false, false>(__VA_ARGS__);                  \
        if (ub_ && !gc_) return fn<14, true, false, true>(__VA_ARGS__);    \
        return fn<14, false, true, true>(__VA_ARGS__);                     \
      default: return fn<16, false, true, true>(__VA_ARGS__);              \
    }                                                                      \
  } while (0)

}  // namespace pgw

using namespace pgw;

// k_coord_pf_od_list's grid (blocks of kBlock lanes): with an empty list (the
// usual step) its time is the dispatch of that many blocks of a 148-KB-LDS,
// 512-register kernel; a non-empty list of c envs takes ceil(c / (grid kBlock))
// grid-stride passes.  PGW_OD_LIST_GRID at load (A/Bs), default kOdListGrid.
constexpr int kOdListGrid = 1 << 30;   // (no cap: one block per 256 list slots)
static int initial_od_list_grid() {
  const char* v = getenv("PGW_OD_LIST_GRID");
  const int g = v ? atoi(v) : 0;
  return g > 0 ? g : kOdListGrid;
}
static const int g_od_list_grid = initial_od_list_grid();
// k_coord_step_od's stores: plain / nontemporal (default) or write-through
// (PGW_STEP_WT=1 at load, A/Bs: measured slower, 21.6 -> 23.2 us)
static bool initial_step_wt() {
  const char* v = getenv("PGW_STEP_WT");
  return v && v[0] == '1';
}
static const bool g_step_wt = initial_step_wt();
static const bool g_step_nolookup = getenv("PGW_STEP_NOLOOKUP") && getenv("PGW_STEP_NOLOOKUP")[0] == '1';
// PGW_STEP_NOP=1 (diagnostics): an empty one-wave kernel between the step's two launches, to time the boundary
static const bool g_step_nop = getenv("PGW_STEP_NOP") && getenv("PGW_STEP_NOP")[0] == '1';
// PGW_STEP_LIST=1 (A/Bs): the two-launch form of the fused step -- the envs
// the table left listed by k_coord_step_od and solved by k_coord_pf_od_list --
// instead of the inline wave solve.  PGW_STEP_NOLIST=1 (diagnostics, with
// PGW_STEP_LIST=1): no list launch -- the listed envs keep their raw rewards
// and unsolved voltages (timing only).
static const bool g_step_list = getenv("PGW_STEP_LIST") && getenv("PGW_STEP_LIST")[0] == '1';
static const bool g_step_nolist = getenv("PGW_STEP_NOLIST") && getenv("PGW_STEP_NOLIST")[0] == '1';
static ODWaveArgs make_wave_args(const PFArgs& a, const ODArgs& o, const pgw_pf_params& pf,
                                 const pgw_pf_tables& t) {
  ODWaveArgs z = {};
  for (int k = 0; k < PGW_PF_MAX_M; ++k) {
    z.sr0[k] = a.sr0[k];
    z.si0[k] = a.si0[k];
    z.fr[k] = a.fr[k];
    z.fi[k] = a.fi[k];
    z.y0r[k] = o.y0r[k];
    z.y0i[k] = o.y0i[k];
    z.esc[k] = o.esc[k];
  }
  z.lo2 = a.lo2;
  z.mn2 = a.mn2;
  z.mx2 = a.mx2;
  z.tol = o.tol;
  z.gamma = o.gamma;
  z.eps = o.eps;
  z.gmax = o.gmax;
  z.gsrc = o.gsrc;
  z.block = t.block;
  z.start = o.start;
  z.rows_V0 = o.rows_V0;
  z.rows_G = o.rows_G;
  z.m = pf.m;
  z.min_iter = o.min_iter;
  z.n_rep = o.n_rep;
  z.n_rows = o.n_rows;
  z.max_iter = o.max_iter;
  z.node_mask = o.node_mask;
  return z;
}
__global__ void k_step_nop(int* p) {
  if (p && threadIdx.x == 1000) *p = 0;
}

// pgw_coord_step / pgw_coord_step_f32
// The agents' half of the coordinated step (k_coord_agents_std or the generic
// k_coord_agents), fp64 buffers.
static int32_t launch_coord_agents(const pgw_coord_params& p, const pgw_coord_step_info& s, int64_t n,
                                   const pgw_coord_buffers& b, double pv_ob, bool std_layout, hipStream_t st) {
  if (std_layout)
    launch_timed(PGW_T_COORD_AGENTS, k_coord_agents_std<pgw_coord_buffers>, dim3(grid_for(n), p.n_agents),
                 dim3(kBlock), st, p, s, n, b, pv_ob, make_std_derived(p));
  else
    launch_timed(PGW_T_COORD_AGENTS, k_coord_agents, dim3(grid_for(n), p.n_agents), dim3(kBlock), st, p, s, n,
                 b);
  return check_launch("k_coord_agents");
}

// The agents' kernel, then the power flow with the coordinated prologue and
// epilogue, on one stream.
template <class Bufs>
static int32_t coord_step(const pgw_coord_params* p, const pgw_pf_params* pf, const pgw_pf_tables* pft,
                          const pgw_coord_step_info* s, int64_t n, const Bufs& b, void* stream) {
  constexpr bool kF32 = std::is_same<Bufs, pgw_coord_buffers_f32>::value;
  PGW_REQUIRE(p && pf && pft && s && n >= 0, "pgw_coord_step: null argument");
  PGW_REQUIRE(p->n_agents >= 1 && p->n_agents <= PGW_MAX_AGENTS, "pgw_coord_step: bad n_agents");
  PGW_REQUIRE(p->n_comp >= 1 && p->n_comp <= 3, "pgw_coord_step: bad n_comp");
  PGW_REQUIRE(b.action.ptr && b.obs.ptr && b.reward && b.agent_power,
              "pgw_coord_step: null buffer");
  PGW_REQUIRE(pft->block, "pgw_coord_step: null PF block");
  PGW_REQUIRE(!pft->load_scale && !pft->U_init, "pgw_coord_step: load_scale / U_init not supported");
  PGW_REQUIRE(pf->m >= 1 && pf->m <= PGW_PF_MAX_M && pf->m == padded_m(pf->m),
              "pgw_coord_step: pf m=%d not padded", pf->m);
  PGW_REQUIRE(pf->n_out >= 1 && p->vv_row >= 0 && p->vv_row < pf->n_out,
              "pgw_coord_step: bad vv_row");
  PGW_REQUIRE(pft->G && pft->V0, "pgw_coord_step: missing G/V0");
  PGW_REQUIRE(pf->max_iter >= 1, "pgw_coord_step: max_iter < 1");
  PGW_REQUIRE(pf->n_ctrl >= 0 && pf->n_ctrl <= PGW_PF_MAX_CTRL, "pgw_coord_step: bad n_ctrl");
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
  const bool std_layout = coord_is_std(*p);
  PGW_REQUIRE(std_layout || !kF32,
              "pgw_coord_step_f32: needs the standard C4 agent layout (building/pv/storage at 0/6/7)");
  if (pft->od) {
    const int32_t rc_od = check_od(*pf, *pft, "pgw_coord_step");
    if (rc_od) return rc_od;
  }
  // PVEnv.get_obs is the same for every env: evaluate it once here
  const double pv_ob = p->pv.rescale ? (2.0 * std::min(std::max(-s->pv_pmax, p->pv.obs_low), p->pv.obs_high)
                                        - (p->pv.obs_low + p->pv.obs_high)) / (p->pv.obs_high - p->pv.obs_low)
                                     : -s->pv_pmax;
  CoordPFArgs c = {};
  c.n_agents = p->n_agents;
  c.coordinated = p->coordinated;
  c.vv_row = p->vv_row;
  for (int a = 0; a < p->n_agents; ++a) c.agent_ctrl[a] = p->agent_ctrl[a];
  c.vv_lo = p->vv_lo;
  c.vv_hi = p->vv_hi;
  c.vv_penalty = p->vv_penalty;
  const PFArgs a = make_pf_args(*pf, *pft);
  if constexpr (!kF32) {
    // OpenDSS rule with the hour's node records and no output row but the
    // coordinated bus: the agents and the table lookup in one launch
    // (k_coord_step_od), then the snap solve of the envs it listed
    // (k_coord_pf_od_list, a small grid that exits at once on an empty list)
    if (pft->od && b.od_list && b.od_count && !g_pf_trace_on.load()) {
      const ODArgs o = make_od_args(*pft->od, pf->max_iter);
      if (std_layout && o.resp_v && o.resp_v_row == 0 && pf->n_out == 1 && p->vv_row == 0) {
        const ODVLook lk = {o.resp_v, o.resp_x0, o.resp_inv_h, o.resp_nseg, g_step_nolookup ? 1 : 0};
        const StepOdArgs sa = {*p, make_wave_args(a, o, *pf, *pft)};
        const dim3 grid((unsigned)((n + 63) / 64)), block(64 * p->n_agents);
        if (!g_step_list) {                         // the one-launch step
          if (g_step_wt)
            launch_timed(PGW_T_COORD_AGENTS, k_coord_step_od<true, true>, grid, block, st, sa, *s, n, b, pv_ob,
                         make_std_derived(*p), c, lk);
          else
            launch_timed(PGW_T_COORD_AGENTS, k_coord_step_od<false, true>, grid, block, st, sa, *s, n, b, pv_ob,
                         make_std_derived(*p), c, lk);
          return check_launch("k_coord_step_od");
        }
        if (g_step_wt)
          launch_timed(PGW_T_COORD_AGENTS, k_coord_step_od<true, false>, grid, block, st, sa, *s, n, b, pv_ob,
                       make_std_derived(*p), c, lk);
        else
          launch_timed(PGW_T_COORD_AGENTS, k_coord_step_od<false, false>, grid, block, st, sa, *s, n, b, pv_ob,
                       make_std_derived(*p), c, lk);
        int32_t rc = check_launch("k_coord_step_od");
        if (rc) return rc;
        if (g_step_nop) hipLaunchKernelGGL(k_step_nop, dim3(1), dim3(64), 0, st, (int*)nullptr);
        if (g_step_nolist) return PGW_OK;
        if (g_od_list_grid >= grid_for(n))
          launch_timed(PGW_T_COORD_PF, k_coord_pf_od_list<14, false>, dim3((unsigned)grid_for(n)),
                       dim3(kBlock), st, c, a, o, *pft, n, b);
        else
          launch_timed(PGW_T_COORD_PF, k_coord_pf_od_list<14, true>, dim3((unsigned)g_od_list_grid),
                       dim3(kBlock), st, c, a, o, *pft, n, b);
        return check_launch("k_coord_pf_od_list");
      }
    }
    // any other step with a list: the next step's count (k_coord_step_od's job) zeroed here
    if (b.od_count) {
      const hipError_t me = hipMemsetAsync(b.od_count + ((b.od_parity & 1) ^ 1), 0, sizeof(int32_t), st);
      PGW_REQUIRE(me == hipSuccess, "pgw_coord_step: od_count reset: %s", hipGetErrorString(me));
    }
  }
  // fp32: env pairs per lane (float2 accesses).  The pair layout measured for
  // fp64 too (19.5 -> 20.2 us), so it is instantiated for fp32 only.
  bool done = false;
  if constexpr (kF32) {
    if (std_layout && pairs_ok(b, n)) {
      launch_timed(PGW_T_COORD_AGENTS, k_coord_agents_std_x2<Bufs>, dim3(grid_for(n / 2), p->n_agents),
                   dim3(kBlock), st, *p, *s, n, b, pv_ob, make_std_derived(*p));
      done = true;
    }
  }
  if (done) {
  } else if (std_layout) {
    launch_timed(PGW_T_COORD_AGENTS, k_coord_agents_std<Bufs>, dim3(grid_for(n), p->n_agents),
                 dim3(kBlock), st, *p, *s, n, b, pv_ob, make_std_derived(*p));
  } else if constexpr (!kF32) {
    launch_timed(PGW_T_COORD_AGENTS, k_coord_agents, dim3(grid_for(n), p->n_agents), dim3(kBlock),
                 st, *p, *s, n, b);
  }
  int32_t rc = check_launch("k_coord_agents");
  if (rc) return rc;
  if (g_step_nop) hipLaunchKernelGGL(k_step_nop, dim3(1), dim3(64), 0, st, (int*)nullptr);
  hipStream_t pst = st;
  if (pft->od) {
    if (g_pf_trace_on.load())
      launch_timed(PGW_T_COORD_PF, k_coord_pf_od<14, Bufs, true>, dim3(grid_for(n)), dim3(kBlock), pst, c, a,
                   make_od_args(*pft->od, pf->max_iter), *pft, n, b);
    else
      launch_timed(PGW_T_COORD_PF, k_coord_pf_od<14, Bufs>, dim3(grid_for(n)), dim3(kBlock), pst, c, a,
                   make_od_args(*pft->od, pf->max_iter), *pft, n, b);
    return check_launch("k_coord_pf_od");
  }
  PGW_PF_DISPATCH(*pf, *pft, launch_coord_pf, c, a, *pft, n, b, pst);
}

// pgw_coord_step_general: the agents' kernel, then the general power flow with
// the coordinated prologue (bus load = agent powers summed in agent order) and
// epilogue (voltage violation, reward -= share) of k_coord_pf.
static int32_t coord_step_general(const pgw_coord_params* p, const pgw_pfg_params* pf,
                                  const pgw_pfg_tables* pft, const pgw_coord_step_info* s, int64_t n,
                                  const pgw_coord_buffers& b, void* stream) {
  PGW_REQUIRE(p && pf && pft && s && n >= 0, "pgw_coord_step_general: null argument");
  PGW_REQUIRE(p->n_agents >= 1 && p->n_agents <= PGW_MAX_AGENTS, "pgw_coord_step_general: bad n_agents");
  PGW_REQUIRE(p->n_comp >= 1 && p->n_comp <= 3, "pgw_coord_step_general: bad n_comp");
  PGW_REQUIRE(b.action.ptr && b.obs.ptr && b.reward && b.agent_power, "pgw_coord_step_general: null buffer");
  PGW_REQUIRE(pf->n_out >= 1 && p->vv_row >= 0 && p->vv_row < pf->n_out, "pgw_coord_step_general: bad vv_row");
  for (int a = 0; a < p->n_agents; ++a)
    PGW_REQUIRE(p->agent_ctrl[a] < pf->n_ctrl, "pgw_coord_step_general: agent_ctrl out of range");
  for (int c = 0; c < p->n_comp; ++c) {
    int k = p->comp_order[c];
    PGW_REQUIRE(k >= 0 && k <= 2, "pgw_coord_step_general: bad comp_order");
    if (k == 0) PGW_REQUIRE(b.x && p->act_bld >= 0 && p->bld.n_obs <= PGW_BLD_MAX_OBS, "pgw_coord_step_general: building");
    if (k == 2) PGW_REQUIRE(b.soc && p->act_bat >= 0, "pgw_coord_step_general: storage");
  }
  if (n == 0) return PGW_OK;
  const double pv_ob = p->pv.rescale ? (2.0 * std::min(std::max(-s->pv_pmax, p->pv.obs_low), p->pv.obs_high)
                                        - (p->pv.obs_low + p->pv.obs_high)) / (p->pv.obs_high - p->pv.obs_low)
                                     : -s->pv_pmax;
  if (b.od_count) {                                // (pgw_coord_buffers.od_count: the next step's list)
    const hipError_t me = hipMemsetAsync(b.od_count + ((b.od_parity & 1) ^ 1), 0, sizeof(int32_t),
                                         (hipStream_t)stream);
    PGW_REQUIRE(me == hipSuccess, "pgw_coord_step_general: od_count reset: %s", hipGetErrorString(me));
  }
  int32_t rc = launch_coord_agents(*p, *s, n, b, pv_ob, coord_is_std(*p), (hipStream_t)stream);
  if (rc) return rc;
  PFGCoord c = {};
  c.agent_power = b.agent_power;
  c.reward = b.reward;
  c.vv = b.vv;
  c.n_agents = p->n_agents;
  c.vv_row = p->vv_row;
  c.coordinated = p->coordinated;
  for (int a = 0; a < p->n_agents; ++a) c.agent_ctrl[a] = p->agent_ctrl[a];
  c.vv_lo = p->vv_lo;
  c.vv_hi = p->vv_hi;
  c.vv_penalty = p->vv_penalty;
  return solve_general(pf, pft, n, nullptr, nullptr, b.v_out, b.iters, c, stream);
}

extern "C" {

int32_t pgw_coord_step_general(const pgw_coord_params* p, const pgw_pfg_params* pf,
                               const pgw_pfg_tables* pft, const pgw_coord_step_info* s, int64_t n,
                               pgw_coord_buffers b, void* stream) {
  return coord_step_general(p, pf, pft, s, n, b, stream);
}

int32_t pgw_pf_padded_m(int32_t m) { return padded_m(m); }

int32_t pgw_voltage_band_penalty(int64_t n, const double* v, double lo, double hi, double scale,
                                 double* out, void* stream) {
  PGW_REQUIRE(v && out && n >= 0, "pgw_voltage_band_penalty: null argument");
  if (n == 0) return PGW_OK;
  hipLaunchKernelGGL(k_band_penalty, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, n, v, lo,
                     hi, scale, out);
  return check_launch("k_band_penalty");
}

int64_t pgw_pf_od_probe_args_size(int32_t n_hours) {
  return n_hours <= 0 ? 0 : (int64_t)n_hours * (int64_t)sizeof(PFArgs);
}

int32_t pgw_pf_od_probe(const pgw_pf_params* p_hours, int32_t n_hours, const pgw_pf_tables* t,
                        const double* start_h, int32_t lanes_per_hour, int64_t n, const double* P,
                        double* J_out, uint64_t* sig_out, int32_t* it_out, void* args_buf, void* stream) {
  PGW_REQUIRE(p_hours && t && t->block && t->od && start_h && P && J_out && sig_out && it_out && args_buf,
              "pgw_pf_od_probe: null argument");
  PGW_REQUIRE(n_hours >= 1 && n >= 0 && lanes_per_hour > 0 && lanes_per_hour % kBlock == 0 &&
              n <= (int64_t)n_hours * lanes_per_hour,
              "pgw_pf_od_probe: n %lld lanes over %d hours of %d (a multiple of %d)", (long long)n, n_hours,
              lanes_per_hour, kBlock);
  std::vector<PFArgs> args(n_hours);
  for (int h = 0; h < n_hours; ++h) {
    const int32_t rc = check_od(p_hours[h], *t, "pgw_pf_od_probe");
    if (rc) return rc;
    PGW_REQUIRE(p_hours[h].m == p_hours[0].m && p_hours[h].n_ctrl == p_hours[0].n_ctrl &&
                p_hours[h].max_iter == p_hours[0].max_iter, "pgw_pf_od_probe: hours differ in shape");
    args[h] = make_pf_args(p_hours[h], *t);
  }
  if (n == 0) return PGW_OK;
  hipStream_t st = (hipStream_t)stream;
  // (the host array is released on return: wait for the copy)
  PGW_REQUIRE(hipMemcpyAsync(args_buf, args.data(), sizeof(PFArgs) * n_hours, hipMemcpyHostToDevice, st) ==
                  hipSuccess && hipStreamSynchronize(st) == hipSuccess,
              "pgw_pf_od_probe: argument upload failed");
  hipLaunchKernelGGL(k_pf_od_probe<14>, dim3(grid_for(n)), dim3(kBlock), 0, st,
                     reinterpret_cast<const PFArgs*>(args_buf), make_od_args(*t->od, p_hours[0].max_iter), *t,
                     start_h, lanes_per_hour, n, P, reinterpret_cast<double2*>(J_out), sig_out, it_out);
  return check_launch("k_pf_od_probe");
}

int32_t pgw_pf_od_resp_fit(int32_t m, int64_t n_pieces, const double* J, const int32_t* idx3,
                           const double* meta, const int32_t* inext, const int32_t* rec, double* out,
                           void* stream) {
  PGW_REQUIRE(m >= 1 && m <= PGW_PF_MAX_M && n_pieces >= 0, "pgw_pf_od_resp_fit: bad m / n_pieces");
  if (n_pieces == 0) return PGW_OK;
  PGW_REQUIRE(J && idx3 && meta && inext && rec && out, "pgw_pf_od_resp_fit: null argument");
  hipLaunchKernelGGL(k_pf_od_resp_fit, dim3(grid_for(n_pieces)), dim3(kBlock), 0, (hipStream_t)stream, m,
                     n_pieces, reinterpret_cast<const double2*>(J), idx3, meta, inext, rec, out);
  return check_launch("k_pf_od_resp_fit");
}

int32_t pgw_pf_od_resp_check(int32_t m, int64_t n, const double* recs, const int32_t* rec, const double* P,
                             const double* J, const int32_t* iq, double* err, void* stream) {
  PGW_REQUIRE(m >= 1 && m <= PGW_PF_MAX_M && n >= 0, "pgw_pf_od_resp_check: bad m / n");
  if (n == 0) return PGW_OK;
  PGW_REQUIRE(recs && rec && P && J && iq && err, "pgw_pf_od_resp_check: null argument");
  hipLaunchKernelGGL(k_pf_od_resp_check, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, m, n, recs,
                     rec, P, reinterpret_cast<const double2*>(J), iq, err);
  return check_launch("k_pf_od_resp_check");
}

int32_t pgw_pf_pred_meta(const pgw_pf_params* p, int32_t n_tables, int32_t n_points,
                         const double* U_pred, const int32_t* sig, pgw_pred_meta* meta,
                         void* stream) {
  PGW_REQUIRE(p && U_pred && sig && meta, "pgw_pf_pred_meta: null argument");
  PGW_REQUIRE(n_tables >= 0 && n_points >= 3, "pgw_pf_pred_meta: need >= 3 grid points");
  PGW_REQUIRE(p->m >= 1 && p->m <= PGW_PF_MAX_M, "pgw_pf_pred_meta: bad m");
  const int64_t total = (int64_t)n_tables * (n_points - 1);
  if (total == 0) return PGW_OK;
  hipLaunchKernelGGL(k_pf_pred_meta, dim3(grid_for(total)), dim3(kBlock), 0, (hipStream_t)stream,
                     *p, n_tables, n_points, U_pred, sig, meta);
  return check_launch("k_pf_pred_meta");
}

int32_t pgw_pf_pred_pack(const pgw_pf_params* p, int32_t n_tables, int32_t n_points,
                         const double* U_grid, double* rec, void* stream) {
  PGW_REQUIRE(p && U_grid && rec, "pgw_pf_pred_pack: null argument");
  PGW_REQUIRE(n_tables >= 0 && n_points >= 3, "pgw_pf_pred_pack: need >= 3 grid points");
  PGW_REQUIRE(p->m >= 1 && p->m <= PGW_PF_MAX_M && p->m == padded_m(p->m),
              "pgw_pf_pred_pack: m=%d not padded", p->m);
  PGW_REQUIRE((reinterpret_cast<uintptr_t>(rec) & 15) == 0, "pgw_pf_pred_pack: rec not 16-byte aligned");
  const int64_t total = (int64_t)n_tables * n_points;
  if (total == 0) return PGW_OK;
  hipStream_t st = (hipStream_t)stream;
  switch (p->m) {
    case 8: hipLaunchKernelGGL(k_pf_pred_pack<8>, dim3(grid_for(total)), dim3(kBlock), 0, st, n_tables, n_points, U_grid, rec); break;
    case 14: hipLaunchKernelGGL(k_pf_pred_pack<14>, dim3(grid_for(total)), dim3(kBlock), 0, st, n_tables, n_points, U_grid, rec); break;
    default: hipLaunchKernelGGL(k_pf_pred_pack<16>, dim3(grid_for(total)), dim3(kBlock), 0, st, n_tables, n_points, U_grid, rec); break;
  }
  return check_launch("k_pf_pred_pack");
}

int32_t pgw_debug_pf_trace(long long* buf) {
  PGW_REQUIRE(hipMemcpyToSymbol(HIP_SYMBOL(g_pf_trace), &buf, sizeof(buf)) == hipSuccess,
              "pgw_debug_pf_trace: hipMemcpyToSymbol failed");
  g_pf_trace_on.store(buf != nullptr);
  return PGW_OK;
}

int64_t pgw_pf_pack_size(int32_t m) { return pf_block_size(m); }

int32_t pgw_pf_pack(const pgw_pf_params* p, const double* W, const double* U0, const double* G0,
                    const double* V0_0, double* out) {
  PGW_REQUIRE(p && W && U0 && out, "pgw_pf_pack: null argument");
  PGW_REQUIRE(p->n_out == 0 || (G0 && V0_0), "pgw_pf_pack: output node 0 row missing");
  const int M = p->m;
  PGW_REQUIRE(M >= 1 && M <= PGW_PF_MAX_M && M == padded_m(M), "pgw_pf_pack: m=%d not padded", M);
  for (int k = 0; k < M; ++k)
    PGW_REQUIRE(p->vbase[k] > 0.0, "pgw_pf_pack: vbase[%d] <= 0", k);
  auto w = [&](int i, int k, int c) { return W[2 * (i * M + k) + c]; };
  double wmax = 0.0, asym = 0.0;
  for (int i = 0; i < M; ++i)
    for (int k = 0; k < M; ++k)
      for (int c = 0; c < 2; ++c) {
        wmax = std::max(wmax, std::fabs(w(i, k, c)));
        asym = std::max(asym, std::fabs(w(i, k, c) - w(k, i, c)));
      }
  // W = -C Z C^T is complex symmetric for a reciprocal network (no phase shifters)
  PGW_REQUIRE(asym <= 1e-12 * wmax, "pgw_pf_pack: W not symmetric (%.3g relative)",
              wmax > 0 ? asym / wmax : asym);
  const int T = M * (M + 1) / 2;
  for (int i = 0; i < M; ++i)
    for (int k = i; k < M; ++k) {
      const double sc = 1.0 / (p->vbase[i] * p->vbase[k]);
      const double wr = 0.5 * (w(i, k, 0) + w(k, i, 0)) * sc, wi = 0.5 * (w(i, k, 1) + w(k, i, 1)) * sc;
      const int e = i * M - i * (i - 1) / 2 + (k - i);
      out[e] = wr;
      out[T + e] = wi;
      out[2 * T + e] = wr + wi;
    }
  const int64_t u0 = 3LL * T;
  for (int k = 0; k < M; ++k) {
    const double ur = U0[2 * k] / p->vbase[k], ui = U0[2 * k + 1] / p->vbase[k];
    out[u0 + k] = ur;
    out[u0 + M + k] = ui;
    out[u0 + 2 * M + k] = ur + ui;
    out[u0 + 3 * M + k] = p->vlow[k] * p->vlow[k];
    out[u0 + 4 * M + k] = p->vmin[k] * p->vmin[k];
    out[u0 + 5 * M + k] = p->vmax[k] * p->vmax[k];
    // output row 0 of the tables, verbatim (already in pu against I'_k)
    out[u0 + 6 * M + k] = G0 ? G0[2 * k] : 0.0;
    out[u0 + 7 * M + k] = G0 ? G0[2 * k + 1] : 0.0;
  }
  out[u0 + 8 * M] = V0_0 ? V0_0[0] : 0.0;
  out[u0 + 8 * M + 1] = V0_0 ? V0_0[1] : 0.0;
  return PGW_OK;
}

}  // extern "C"

// pgw_pf_solve / pgw_pf_solve_f32 (IO: the per-env buffers' storage type)
template <class IO>
static int32_t pf_solve(const pgw_pf_params* p, const pgw_pf_tables* t, int64_t n, const IO* ctrl_p,
                        const IO* ctrl_q, IO* v_out, int32_t* iters, void* stream) {
  PGW_REQUIRE(p && t && t->block && n >= 0, "pgw_pf_solve: null argument");
  PGW_REQUIRE(p->m >= 1 && p->m <= PGW_PF_MAX_M && p->m == padded_m(p->m),
              "pgw_pf_solve: m=%d not padded (pgw_pf_padded_m)", p->m);
  PGW_REQUIRE(p->n_ctrl >= 0 && p->n_ctrl <= PGW_PF_MAX_CTRL, "pgw_pf_solve: bad n_ctrl");
  PGW_REQUIRE(p->n_out == 0 || (t->G && t->V0), "pgw_pf_solve: missing G/V0");
  PGW_REQUIRE(p->n_out == 0 || v_out || t->v_min_out || t->v_max_out,
              "pgw_pf_solve: n_out > 0 but no output (v_out, v_min_out, v_max_out all NULL)");
  PGW_REQUIRE(p->max_iter >= 1, "pgw_pf_solve: max_iter < 1");
  if (t->od) {
    const int32_t rc = check_od(*p, *t, "pgw_pf_solve");
    if (rc) return rc;
  }
  if (n == 0) return PGW_OK;
  const PFArgs a = make_pf_args(*p, *t);
  if (t->od) {
    launch_timed(PGW_T_PF_SOLVE, k_pf_solve_od<14, IO>, dim3(grid_for(n)), dim3(kBlock), (hipStream_t)stream, a,
                 make_od_args(*t->od, p->max_iter), *t, n, ctrl_p, ctrl_q, v_out, iters);
    return check_launch("k_pf_solve_od");
  }
  PGW_PF_DISPATCH(*p, *t, launch_pf_solve, a, *t, n, ctrl_p, ctrl_q, v_out, iters, (hipStream_t)stream);
}

extern "C" {

int32_t pgw_pf_solve(const pgw_pf_params* p, const pgw_pf_tables* t, int64_t n,
                     const double* ctrl_p, const double* ctrl_q, double* v_out, int32_t* iters,
                     void* stream) {
  return pf_solve(p, t, n, ctrl_p, ctrl_q, v_out, iters, stream);
}

int32_t pgw_pf_solve_f32(const pgw_pf_params* p, const pgw_pf_tables* t, int64_t n,
                         const float* ctrl_p, const float* ctrl_q, float* v_out, int32_t* iters,
                         void* stream) {
  return pf_solve(p, t, n, ctrl_p, ctrl_q, v_out, iters, stream);
}

int32_t pgw_coord_step(const pgw_coord_params* p, const pgw_pf_params* pf, const pgw_pf_tables* pft,
                       const pgw_coord_step_info* s, int64_t n, pgw_coord_buffers b, void* stream) {
  return coord_step(p, pf, pft, s, n, b, stream);
}

int32_t pgw_coord_step_f32(const pgw_coord_params* p, const pgw_pf_params* pf,
                           const pgw_pf_tables* pft, const pgw_coord_step_info* s, int64_t n,
                           pgw_coord_buffers_f32 b, void* stream) {
  return coord_step(p, pf, pft, s, n, b, stream);
}

}  // extern "C"
