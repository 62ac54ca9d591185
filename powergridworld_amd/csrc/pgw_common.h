// Shared device helpers for libpgw (gfx950).  Built with -ffp-contract=off so
// every expression rounds exactly as the reference's NumPy fp64 arithmetic;
// the power-flow kernel opts into fma() explicitly where it wants it.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pgw.h"

namespace pgw {

// ---------------------------------------------------------------- errors
void set_error(const char* fmt, ...);
int32_t check_launch(const char* what);

#define PGW_REQUIRE(cond, ...)            \
  do {                                    \
    if (!(cond)) {                        \
      ::pgw::set_error(__VA_ARGS__);      \
      return PGW_ERR_ARG;                 \
    }                                     \
  } while (0)

// Sampled launch timing (pgw_timing.hip).  A sampled launch goes through
// hipExtLaunchKernelGGL with a start/stop event pair, whose timestamps come
// from the kernel's own dispatch (the same interval rocprofv3 reports);
// every other launch is a plain hipLaunchKernelGGL.
struct TimingSlot {
  hipEvent_t start = nullptr, stop = nullptr;
};
TimingSlot timing_begin(int kernel);
void timing_commit(int kernel, const TimingSlot& s);

template <typename K, typename... A>
inline void launch_timed(int id, K kernel, dim3 grid, dim3 block, hipStream_t st, A... args) {
  const TimingSlot s = timing_begin(id);
  if (s.start) {
    hipExtLaunchKernelGGL(kernel, grid, block, 0, st, s.start, s.stop, 0, args...);
    timing_commit(id, s);
  } else {
    hipLaunchKernelGGL(kernel, grid, block, 0, st, args...);
  }
}

// A kernel's FIRST by-value struct argument read in place from the kernarg
// segment (constant address space: scalar loads, dynamic indices included).
// Naming the by-value parameter itself makes clang copy it into a private
// alloca that the optimizer must then remove; in the big fused-step kernels it
// did not always (k_ma_step<false> copied its 3.2 KB argument struct to
// scratch per lane: a PV-only step took 38.9 us instead of 5.1).
#ifdef __HIP_DEVICE_COMPILE__
#define PGW_KERNARG0(T) (*(const T*)__builtin_amdgcn_kernarg_segment_ptr())
#else
#define PGW_KERNARG0(T) (*(const T*)nullptr)
#endif

constexpr int kBlock = 256;   // 4 waves of 64

// The general power flow (pgw_pf_general.hip) with an optional coordinated
// prologue / epilogue (pgw_coord_step_general): bus load = sum of the agents'
// powers in agent order (multiagent_env.py:171-181), and
// CoordinatedMultiBuildingControlEnv.reward_transform (train.py:51-88) on the
// common-bus voltage row.  agent_power == nullptr: a plain solve (ctrl_p/q).
struct PFGCoord {
  const double* agent_power;   // n_agents x n
  double* reward;              // n_agents x n
  double* vv;                  // n (nullable)
  int32_t n_agents, vv_row, coordinated, pad_;
  int32_t agent_ctrl[PGW_MAX_AGENTS];
  double vv_lo, vv_hi, vv_penalty;
};
int32_t solve_general(const pgw_pfg_params* p, const pgw_pfg_tables* t, int64_t n, const double* cp,
                      const double* cq, double* v_out, int32_t* iters, const PFGCoord& c, void* stream);

inline unsigned grid_for(int64_t n) {
  return static_cast<unsigned>((n + kBlock - 1) / kBlock);
}

// ---------------------------------------------------------------- numpy semantics
// np.clip(x, lo, hi) == minimum(maximum(x, lo), hi), NaN-propagating.
__device__ __forceinline__ double clip(double x, double lo, double hi) {
  double y = (x < lo) ? lo : x;
  return (y > hi) ? hi : y;
}

// The same result (lo <= hi) from v_max/v_min, which take the bounds as SGPR
// operands: x itself whenever it equals the clamped value (in range, or equal
// to a bound -- also keeps x's sign of zero) or is NaN, else the bound.
__device__ __forceinline__ double clip_fast(double x, double lo, double hi) {
  const double r = fmin(fmax(x, lo), hi);
  return (r == x || x != x) ? x : r;
}

// x / d correctly rounded, from r = RN(1/d): one multiply and two residual
// corrections (Markstein: r correctly rounded and q1 faithful => q2 = RN(x/d)),
// i.e. bit-identical to the IEEE quotient -- checked against it by
// tests/test_cpu_host.py::test_exact_division.  Zero numerators take x * r (the
// residual step would turn -0 into +0).  For finite x and normal d only.
__device__ __forceinline__ double exact_div(double x, double d, double r) {
  const double q0 = x * r;
  const double q1 = fma(fma(-d, q0, x), r, q0);
  const double q2 = fma(fma(-d, q1, x), r, q1);
  return x == 0.0 ? q0 : q2;
}

// gridworld/utils.py:9-24
__device__ __forceinline__ double to_scaled(double x, double lo, double hi) {
  x = clip(x, lo, hi);
  return (2.0 * x - (lo + hi)) / (hi - lo);
}

// The reference's to_raw warning condition (utils.py:36): y outside
// [-1 - eps, 1 + eps], NaN included.  oob_note counts one warning (PGW_OOB in
// pgw.h): the atomic is taken only by the lanes that would have warned.
__device__ __forceinline__ bool oob_bad(double y) {
  return !(y >= -1.0 - PGW_OOB_EPS && y <= 1.0 + PGW_OOB_EPS);
}
__device__ __forceinline__ void oob_note(uint64_t* c, bool bad) {
  if (c != nullptr && bad) atomicAdd(reinterpret_cast<unsigned long long*>(c), 1ull);
}

// gridworld/utils.py:27-43 (the warning: oob_bad / oob_note at the call sites)
__device__ __forceinline__ double to_raw(double y, double lo, double hi) {
  y = clip(y, -1.0, 1.0);
  return (y * (hi - lo) + (hi + lo)) / 2.0;
}

// Python's max(a, b) for floats (first argument wins ties / NaN on the right).
__device__ __forceinline__ double pymax(double a, double b) { return (b > a) ? b : a; }
__device__ __forceinline__ double pymin(double a, double b) { return (b < a) ? b : a; }

// Action element (e, j) of a pgw_mat or pgw_matf; fp32 values are widened to
// fp64 (exactly).  Every caller loads actions: they are read once per step, so
// the load is nontemporal (C4: profiles/r02/act_nt.txt).
template <class Mt>
__device__ __forceinline__ double ld(const Mt& m, int64_t e, int j) {
  return (double)__builtin_nontemporal_load(m.ptr + e * m.s_env + (int64_t)j * m.s_dim);
}
// Observation stores are write-once streams for the policy: nontemporal, so
// they do not evict the state the next step re-reads (k_coord_agents_std
// 21.4 -> 19.6 us at C4, profiles/r01/nt_stores.txt).
// fp32 storage (the *_f32 entries): the fp64 value is rounded once, here.
__device__ __forceinline__ void st_obs(double* p, double v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ void st_obs(float* p, double v) { __builtin_nontemporal_store((float)v, p); }
// Write-through store (global_store ... sc1, a relaxed agent-scope store): the
// line leaves the XCD's L2 with the store instead of staying there dirty.  A
// kernel boundary writes back whatever its predecessor left dirty (about
// bytes / 6 TB/s, MI355X_MICROARCH.md "boundary"), so a step kernel whose
// outputs (~100 MB, far beyond the 32 MB of L2) are all write-through leaves
// the next launch a clean boundary.
template <class T>
__device__ __forceinline__ void st_wt(T* p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <class Mt>
__device__ __forceinline__ void st(const Mt& m, int64_t e, int j, double v) {
  st_obs(m.ptr + e * m.s_env + (int64_t)j * m.s_dim, v);
}

// ---------------------------------------------------------------- battery
// energy_storage_env.py:100-157.  Returns the (validated) power; updates soc.
// `div(x, which)` divides x by eta_d (which 0) or dt_h (which 1).
template <class Div>
__device__ __forceinline__ double battery_step_impl(const pgw_battery_params& p, double a, double& soc,
                                                    Div&& div) {
  if (p.rescale) {
    oob_note(p.oob, oob_bad(a));
    a = to_raw(a, -1.0, 1.0);
  }
  double power = a * p.max_power;
  // validate_power :112-126 (the clamps omit the efficiencies, as in the reference)
  if (power > 0.0) {
    if (soc - div(power * p.dt_h, 0) < p.soc_min)
      power = div(pymax(soc - p.soc_min, 0.0), 1);
  } else if (power < 0.0) {
    if (soc - p.eta_c * power * p.dt_h > p.soc_max)
      power = -div(pymax(p.soc_max - soc, 0.0), 1);
  }
  if (power < 0.0) {
    soc = soc - p.eta_c * power * p.dt_h;
    soc = pymin(soc, p.soc_max);
  } else if (power > 0.0) {
    soc = soc - div(power * p.dt_h, 0);
    soc = pymax(soc, p.soc_min);
  }
  return power;
}

__device__ __forceinline__ double battery_step(const pgw_battery_params& p, double a, double& soc) {
  return battery_step_impl(p, a, soc, [&](double x, int w) { return x / (w ? p.dt_h : p.eta_d); });
}

// The same step with the divisions done by exact_div from host reciprocals
// (bit-identical results).
__device__ __forceinline__ double battery_step_rcp(const pgw_battery_params& p, double a, double& soc,
                                                   double rcp_eta_d, double rcp_dt_h) {
  return battery_step_impl(p, a, soc, [&](double x, int w) {
    return w ? exact_div(x, p.dt_h, rcp_dt_h) : exact_div(x, p.eta_d, rcp_eta_d);
  });
}

__device__ __forceinline__ double battery_obs(const pgw_battery_params& p, double soc) {
  return p.rescale ? to_scaled(soc, p.soc_min, p.soc_max) : soc;
}

// ---------------------------------------------------------------- PV
__device__ __forceinline__ double pv_obs(const pgw_pv_params& p, double pmax) {
  double raw = -pmax;
  return p.rescale ? to_scaled(raw, p.obs_low, p.obs_high) : raw;
}

__device__ __forceinline__ double pv_real_power(const pgw_pv_params& p, double a, double pmax) {
  if (p.rescale) {
    oob_note(p.oob, oob_bad(a));
    a = to_raw(a, 0.0, 1.0);
  }
  return a * (-pmax);
}

// ---------------------------------------------------------------- building
struct BuildingExt {
  double bus_v, min_v, max_v, p_set;
};

__device__ __forceinline__ BuildingExt building_ext(const pgw_building_ext& x, int64_t e) {
  BuildingExt r;
  r.bus_v = x.bus_voltage ? x.bus_voltage[e] : 1.0;
  double dflt = x.bus_voltage ? r.bus_v : 1.0;       // five_zone_rom_env.py:260-262
  r.min_v = x.min_voltage ? x.min_voltage[e] : dflt;
  r.max_v = x.max_voltage ? x.max_voltage[e] : dflt;
  r.p_set = x.p_setpoint ? x.p_setpoint[e] : __builtin_huge_val();
  return r;
}

// u-vector (dynamics.py:12-41) and state update (:44-55) for all zones.
// action == nullptr: reset form (u_pos[7] = q_cool).
__device__ __forceinline__ void building_state_update(const pgw_building_params& p,
                                                      const pgw_building_exo& ex,
                                                      const double T[5], const double* act,
                                                      double x[5]) {
  double u[5][4];
#pragma unroll
  for (int z = 0; z < 5; ++z) {
    double upos[8];
    upos[0] = ex.T_oa - T[z];
    upos[1] = ex.q_solar[z];
    upos[2] = ex.q_int[z];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // neighbour id is uniform (kernel argument): select with a constant-index switch
      int y = p.nbr[z][i];
      double ty = (y == 0) ? T[0] : (y == 1) ? T[1] : (y == 2) ? T[2] : (y == 3) ? T[3] : T[4];
      upos[3 + i] = ty - T[z];
    }
    upos[7] = act ? act[z] * (act[5] - T[z]) : ex.q_cool[z];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int s = p.sel[z][j];
      double v = upos[0];
#pragma unroll
      for (int k = 1; k < 8; ++k) v = (s == k) ? upos[k] : v;
      u[z][j] = v;
    }
  }
#pragma unroll
  for (int z = 0; z < 5; ++z) {
    double bu = p.B[z][0] * u[z][0];
    bu = bu + p.B[z][1] * u[z][1];
    bu = bu + p.B[z][2] * u[z][2];
    bu = bu + p.B[z][3] * u[z][3];
    x[z] = p.A[z] * x[z] + bu;
  }
}

// get_p_consumed (dynamics.py:106-114)
// s^3 correctly rounded (compensated: both products' rounding errors via fma).
// The reference's s**3 is glibc pow(s, 3.0), which is within ~0.502 ulp but not
// correctly rounded: the two differ by one ulp in ~0.1% of inputs (checked
// against exact rationals; the cube was the correctly rounded one each time).
__device__ __forceinline__ double cube_rn(double s) {
  const double p = s * s, e1 = fma(s, s, -p);
  const double q = p * s, e2 = fma(p, s, -q);
  return q + fma(e1, s, e2);
}

__device__ __forceinline__ double building_p_consumed(const double act[6], double T_oa) {
  double s = (((act[0] + act[1]) + act[2]) + act[3]) + act[4];
  double fan = 0.0076 * cube_rn(s) + 4.8865;
  double chiller = pymax(0.0, s * (T_oa - act[5]));
  return fan + chiller;
}

// FiveZoneROMThermalEnergyEnv.step_reward (five_zone_rom_env.py:315-335);
// e = -p_cons / 12 (passed in so a caller can divide by reciprocal).
__device__ __forceinline__ double building_reward(const pgw_building_params& p, const double T[5],
                                                  double lb, double ub, double p_cons, double e) {
  (void)p_cons;
  double c = 0.0;
#pragma unroll
  for (int z = 0; z < 5; ++z) {
    double up = T[z] - ub, lo = lb - T[z];
    double m = pymax(pymax(up, lo), 0.0);
    c = c + m * m;
  }
  c = -c;
  return p.alpha * e * 0.5 + (1.0 - p.alpha) * c;
}
__device__ __forceinline__ double building_reward(const pgw_building_params& p, const double T[5],
                                                  double lb, double ub, double p_cons) {
  return building_reward(p, T, lb, ub, p_cons, -p_cons / 12.0);
}

// get_obs (five_zone_rom_env.py:228-283): values in state-dict order, bounds in
// make_obs_space order (exactly as the reference zips them).
__device__ __forceinline__ double building_obs_value(int var, const double T[5],
                                                     const pgw_building_exo& ex, double p_cons,
                                                     const BuildingExt& xv) {
  if (var < 5) {
    return (var == 0) ? T[0] : (var == 1) ? T[1] : (var == 2) ? T[2] : (var == 3) ? T[3] : T[4];
  }
  if (var < 10) {
    int z = var - 5;
    double t = (z == 0) ? T[0] : (z == 1) ? T[1] : (z == 2) ? T[2] : (z == 3) ? T[3] : T[4];
    return t - ex.comfort_ub;
  }
  if (var < 15) {
    int z = var - 10;
    double t = (z == 0) ? T[0] : (z == 1) ? T[1] : (z == 2) ? T[2] : (z == 3) ? T[3] : T[4];
    return ex.comfort_lb - t;
  }
  switch (var) {
    case PGW_BV_COMFORT_LOWER: return ex.comfort_lb;
    case PGW_BV_COMFORT_UPPER: return ex.comfort_ub;
    case PGW_BV_OUTDOOR_TEMP: return ex.T_oa;
    case PGW_BV_P_CONSUMED: return p_cons;
    case PGW_BV_TIME_OF_DAY: return ex.time_of_day;
    case PGW_BV_BUS_VOLTAGE: return xv.bus_v;
    case PGW_BV_MIN_VOLTAGE: return xv.min_v;
    case PGW_BV_MAX_VOLTAGE: return xv.max_v;
    default: return xv.p_set;
  }
}

template <typename Store>
__device__ __forceinline__ void building_write_obs(const pgw_building_params& p, const double T[5],
                                                   const pgw_building_exo& ex, double p_cons,
                                                   const BuildingExt& xv, Store store) {
  // unrolled to constant indices: a loop bound by n_obs indexed the by-value
  // params dynamically, which made the compiler copy the whole kernel-argument
  // struct to scratch (k_ma_step<false>: 3.2 KB per lane)
#pragma unroll
  for (int j = 0; j < PGW_BLD_MAX_OBS; ++j) {
    if (j >= p.n_obs) break;
    double v = building_obs_value(p.obs_var[j], T, ex, p_cons, xv);
    v = clip(v, p.obs_low[j], p.obs_high[j]);
    if (p.rescale) v = to_scaled(v, p.obs_low[j], p.obs_high[j]);
    store(j, v);
  }
}

// ---------------------------------------------------------------- std building
// The reference's default 5-zone building (state_space_model.p input_sel_list
// [1,8,7,2] / [1,8,6,2] and neighbours, defaults.py:2-10 observation config)
// with the selections as compile-time indices and the divisions by host
// reciprocals (exact_div): the same IEEE results as the generic functions
// above, op for op, in far fewer instructions.  k_coord_agents_std
// (pgw_pf.hip) is the same arithmetic for the C4 agent.
struct BldDerived {
  double act_rng[6], act_sum[6];                 // actions: hi - lo, hi + lo
  double obs_sum[15], obs_rng[15], obs_rcp[15];  // obs: lo + hi, hi - lo, 1 / (hi - lo)
};

inline BldDerived make_bld_derived(const pgw_building_params& p) {
  BldDerived d = {};
  for (int j = 0; j < 6; ++j) {
    d.act_rng[j] = p.act_high[j] - p.act_low[j];
    d.act_sum[j] = p.act_high[j] + p.act_low[j];
  }
  for (int j = 0; j < 15; ++j) {
    d.obs_sum[j] = p.obs_low[j] + p.obs_high[j];
    d.obs_rng[j] = p.obs_high[j] - p.obs_low[j];
    d.obs_rcp[j] = 1.0 / d.obs_rng[j];
  }
  return d;
}

inline bool bld_is_std(const pgw_building_params& p) {
  static const int sel[5][4] = {{0, 7, 6, 1}, {0, 7, 6, 1}, {0, 7, 5, 1}, {0, 7, 5, 1}, {0, 7, 5, 1}};
  static const int nbr[5][4] = {{1, 2, 3, 4}, {0, 2, 3, 4}, {0, 1, 3, 4}, {0, 1, 2, 4}, {0, 1, 2, 3}};
  if (p.n_obs != 15) return false;
  for (int z = 0; z < 5; ++z)
    for (int j = 0; j < 4; ++j)
      if (p.sel[z][j] != sel[z][j] || p.nbr[z][j] != nbr[z][j]) return false;
  for (int j = 0; j < 15; ++j)
    if (p.obs_var[j] != 5 + j) return false;
  return true;
}

// One std building step (five_zone_rom_env.py:183-225 + the thermal-energy
// reward :315-335): av = the 6 actions as given (rescaled if p.rescale), xs =
// x_k in/out.  Returns p_consumed; `reward` = the fresh reward; obs slot j goes
// to store(j, value).
struct NoStamp {
  __device__ void operator()(int) const {}
};
template <class Store, class Stamp = NoStamp>
__device__ __forceinline__ double bld_std_step(const pgw_building_params& B, const BldDerived& d,
                                               const pgw_building_exo& ex, const pgw_building_exo& exn,
                                               double (&av)[6], double (&xs)[5], double& reward,
                                               Store&& store, Stamp&& stamp = Stamp()) {
  double T[5];
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 6; ++j) {   // to_raw (utils.py:27-43) with host (hi - lo), (hi + lo)
    bad = bad || oob_bad(av[j]);
    av[j] = B.rescale ? (clip_fast(av[j], -1.0, 1.0) * d.act_rng[j] + d.act_sum[j]) * 0.5 : av[j];
  }
  if (B.rescale) oob_note(B.oob, bad);
#pragma unroll
  for (int z = 0; z < 5; ++z) T[z] = B.C[z] * xs[z] + B.mean[z];
  stamp(3);                        // (debug trace: the loads have arrived)
#pragma unroll
  for (int z = 0; z < 5; ++z) {
    const int nz = z < 2 ? 4 : (z == 2 ? 3 : 2);
    const double u0 = ex.T_oa - T[z];
    const double u1 = av[z] * (av[5] - T[z]);
    const double u2 = T[nz] - T[z];
    const double u3 = ex.q_solar[z];
    double bu = B.B[z][0] * u0;
    bu = bu + B.B[z][1] * u1;
    bu = bu + B.B[z][2] * u2;
    bu = bu + B.B[z][3] * u3;
    xs[z] = B.A[z] * xs[z] + bu;   // T still holds the pre-step temps
  }
#pragma unroll
  for (int z = 0; z < 5; ++z) T[z] = B.C[z] * xs[z] + B.mean[z];
  const double pc = building_p_consumed(av, ex.T_oa);
  reward = building_reward(B, T, exn.comfort_lb, exn.comfort_ub, pc, exact_div(-pc, 12.0, 1.0 / 12.0));
  stamp(7);                        // (debug trace: state, power and reward done)
  const double lb = exn.comfort_lb, ub = exn.comfort_ub;
  // (the rescale test hoisted out of the loop: a branch per slot kept the
  // compiler from reading the next slots' bounds ahead -- two waited LDS
  // round trips per slot when the parameters are staged in LDS)
  auto obs_value = [&](int j) {
    return j < 5 ? T[j] - ub : j < 10 ? lb - T[j - 5] : j == 10 ? lb
         : j == 11 ? ub : j == 12 ? exn.T_oa : j == 13 ? pc : exn.time_of_day;
  };
  if (B.rescale) {
#pragma unroll
    for (int j = 0; j < 15; ++j) {
      const double c = clip_fast(obs_value(j), B.obs_low[j], B.obs_high[j]);
      store(j, exact_div(2.0 * c - d.obs_sum[j], d.obs_rng[j], d.obs_rcp[j]));
    }
  } else {
#pragma unroll
    for (int j = 0; j < 15; ++j) store(j, clip_fast(obs_value(j), B.obs_low[j], B.obs_high[j]));
  }
  return pc;
}

}  // namespace pgw
