// Home-Steward house: the whole HSMultiComponentEnv step
// per env in one thread.  The reference passes a per-step resource state
// (meta_state: PV / battery / grid power still available, their costs) from
// component to component (gridworld/base_hs.py:114-180); here that state lives
// in registers and the components run in chain order.  Every expression
// follows the reference's operation order (built with -ffp-contract=off), and
// Python's min/max/round semantics are spelled out (pgw_common.h pymin/pymax).
#include <cmath>

#include "pgw_common.h"

namespace pgw {

// meta_state's resource entries (pv_cost and es_cost are always 0: nothing sets
// pv_cost, HSEnergyStorageEnv.step sets es_cost = 0, energy_storage_env_hs.py:233)
struct HSMeta {
  double pv, es, grid;
};

struct HSState {
  double soc, soc_cost, delta_cost, ev_cost, dev_cost;
  double rp[4];        // real power of each chain slot
  double rew_ev, rew_dev;
};

// One chain slot's step_meta record (PGW_HS_META_FIELDS in pgw.h); off = NULL.
struct HSRec {
  double* p;
  int64_t n, e;
  __device__ __forceinline__ void put(int f, double v) const {
    if (p) p[(int64_t)f * n + e] = v;
  }
  // cost, reward, action, solar / es / grid power consumed
  __device__ __forceinline__ void common(double cost, double rew, double a, double sc, double bc,
                                         double gc) const {
    put(0, cost); put(1, rew); put(2, a); put(3, sc); put(4, bc); put(5, gc);
  }
};

// HSPVEnv (pv_profile_env_hs.py:96-160): obs before the advance; the curtailed
// power a * data[index] becomes meta_state pv_power (rew_meta, :146).
// Grid-aware (:81-85, 110-111): min_voltage appended to the obs, box (0.9, 1.1).
__device__ __forceinline__ void hs_pv(const pgw_hs_params& p, const pgw_hs_step_info& s, int rescale,
                                      bool reset, double a, double vmin, HSMeta& M, double& rp, double* ob,
                                      const HSRec& R) {
  ob[0] = rescale ? to_scaled(-s.pv_avail, p.pv_obs_low, 0.0) : -s.pv_avail;
  ob[1] = rescale ? to_scaled(vmin, 0.9, 1.1) : vmin;
  if (reset) {
    M.pv = s.pv_avail;   // get_obs meta pv_power (:118-121)
    return;
  }
  if (rescale) {
    oob_note(p.oob, oob_bad(a));
    a = to_raw(a, p.pv_act_low, p.pv_act_high);
  }
  rp = a * s.pv_avail;
  M.pv = rp;
  R.common(0.0, 0.0, a, s.pv_avail, 0.0, 0.0);   // :151-155, 162-170
  R.put(6, s.pv_avail);
  R.put(7, rp);
}

// HSEnergyStorageEnv.step (energy_storage_env_hs.py:189-270) incl. validate_power (:100-131)
__device__ __forceinline__ double hs_storage_reward(const pgw_hs_params& p, const HSMeta& M, const HSState& S,
                                                    double rp, double* cost_out = nullptr);

__device__ __forceinline__ void hs_storage(const pgw_hs_params& p, const pgw_hs_step_info& s, int rescale,
                                           double a, HSMeta& M, HSState& S, double& rp, const HSRec& R) {
  const double pv_cap = M.pv, grid_cap = M.grid;
  double sc = 0.0, gc = 0.0;
  if (rescale) {
    oob_note(p.oob, oob_bad(a));
    a = to_raw(a, -1.0, 1.0);
  }
  double power = a * p.max_power;
  if (power > 0.0) {
    double delta = power * p.dt_h / p.eta_d;
    if (S.soc <= p.soc_min) {
      power = 0.0;
    } else if (S.soc - delta < p.soc_min) {
      delta = S.soc - p.soc_min;
      power = delta / p.dt_h * p.eta_d;
    }
  } else if (power < 0.0) {
    double delta = -(power * p.dt_h * p.eta_c);
    if (S.soc >= p.soc_max) {
      power = 0.0;
    } else if (S.soc + delta > p.soc_max) {
      delta = p.soc_max - S.soc;
      power = -(delta / p.dt_h / p.eta_c);
    }
  }
  if (power == 0.0) {
    S.delta_cost = 0.0;
    M.es = 0.0;
  } else if (power < 0.0) {
    // charging: PV first, then the grid; weighted cost of the charge (:213-236)
    const double dS = p.eta_c * power * p.dt_h;
    sc = pymin(-power, M.pv);
    gc = pymin(M.grid, -power - sc);
    S.delta_cost = (0.0 * sc + s.grid_cost * gc) / (sc + gc);
    S.soc_cost = (S.soc * S.soc_cost - dS * S.delta_cost) / (S.soc - dS);
    S.soc = S.soc - dS;
    S.soc = pymin(S.soc, p.soc_max);
    M.pv = pymax(0.0, M.pv - sc);
    M.grid = pymax(0.0, M.grid - gc);
    M.es = 0.0;
  } else if (power > 0.0) {
    const double dS = power * p.dt_h / p.eta_d;
    S.soc = pymax(S.soc - dS, p.soc_min);
    M.es = power;
  }
  rp = -power;
  if (R.p) {   // the step's own step_reward, with the meta_state it leaves (:254-265)
    double cost;
    const double rew = hs_storage_reward(p, M, S, rp, &cost);
    R.common(cost, rew, a, sc, 0.0, gc);
    R.put(6, S.soc);
    R.put(7, power);
    R.put(8, pv_cap - sc);
    R.put(9, grid_cap - gc);
    R.put(10, M.es);
  }
}

// the storage's step_reward, evaluated by the house with the FINAL meta_state
// (base_hs.py:163 -> energy_storage_env_hs.py:156-187)
__device__ __forceinline__ double hs_storage_reward(const pgw_hs_params& p, const HSMeta& M, const HSState& S,
                                                    double rp, double* cost_out) {
  const double cost = (rp < 0.0) ? 0.0 : S.delta_cost * p.eta_c * rp * p.dt_h;
  if (cost_out) *cost_out = cost;
  double r = -cost;
  if (M.pv > 0.0 && M.es > 0.0 && S.soc < p.soc_max) r = r - p.max_storage_cost * (p.soc_max - S.soc);
  return r;
}

// HSEVChargingEnv.step (ev_charging_env_hs.py:182-326); reset runs it with the
// action-less default (:144, 185-187).  Vehicles in ascending index order, as
// the reference's set iteration of small ints.
__device__ __forceinline__ void hs_ev(const pgw_hs_params& p, const pgw_hs_step_info& s, int rescale,
                                      bool reset, double a, int64_t n, int64_t e, const pgw_hs_buffers& b,
                                      HSMeta& M, HSState& S, double& rp, double* ob, const HSRec& R) {
  if (reset) a = 0.0;                                   // _action_space.low
  if (rescale) {
    oob_note(p.oob, oob_bad(a));
    a = to_raw(a, 0.0, 1.0);
  }
  const double kwh = a * p.ev_rate * p.ev_hours_per_step;
  uint64_t prev = reset ? 0ull : b.ev_charging[e], now = 0ull;
  double demand = 0.0, consumed = 0.0, dsum = 0.0, unserved = 0.0;
  int nact = 0, dcnt = 0, ndep = 0;
  for (int v = 0; v < p.n_veh; ++v) {
    double* rq = b.ev_req + (int64_t)v * n + e;
    const double r = reset ? p.ev_req0[v] : *rq;
    const bool active = ((s.ev_window >> v) & 1ull) && (r > 0.0);
    double r_new = r;
    if (active) {
      now |= 1ull << v;
      ++nact;
      demand = demand + r;
      const double tl = (p.ev_end_park[v] - s.ev_time) / 60.0;
      if (tl > 0.0) {
        dsum = dsum + pymax(0.0, p.ev_rate - r / tl);
        ++dcnt;
        const double ch = pymin(kwh, r);
        r_new = r - ch;
        consumed = consumed + ch;
      }
    } else if ((prev >> v) & 1ull) {
      unserved = unserved + r;                          // departed (:260-263)
      ++ndep;
    }
    *rq = r_new;
  }
  b.ev_charging[e] = now;
  double st[7];
  st[0] = s.ev_next_time;
  st[1] = p.ev_mult * (double)nact;
  st[2] = p.ev_mult * consumed;
  st[3] = p.ev_mult * demand;
  st[4] = dcnt ? dsum / (double)dcnt : 0.0;
  st[5] = unserved;
  rp = p.ev_mult * consumed;
  const double power = rp * p.ev_steps_per_hour;
  const double pv_cap = M.pv, es_cap = M.es, grid_cap = M.grid;
  double sc = 0.0, bc = 0.0, gc = 0.0;
  if (power == 0.0 || a == 0.0) {
    S.ev_cost = 0.0;
  } else {
    // PV first, then the battery or the grid, whichever is cheaper (:285-313)
    sc = pymin(power, M.pv);
    if (0.0 < s.grid_cost) {
      bc = pymin(M.es, power - sc);
      gc = pymin(M.grid, power - sc - bc);
    } else {
      gc = pymin(M.grid, power - sc);
      bc = pymin(M.es, power - sc - gc);
    }
    const double sum = sc + gc + bc;
    if (sum > 0.0) S.ev_cost = (0.0 * sc + s.grid_cost * gc + 0.0 * bc) / sum;
    // reset's step works on a copy of the kwargs: its draws are not passed on
    if (!reset) {
      M.pv = pymax(0.0, M.pv - sc);
      M.es = pymax(0.0, M.es - bc);
      M.grid = pymax(0.0, M.grid - gc);
    }
  }
  st[6] = S.ev_cost;
#pragma unroll
  for (int j = 0; j < 7; ++j) ob[j] = rescale ? to_scaled(st[j], p.ev_obs_low[j], p.ev_obs_high[j]) : st[j];
  // step_reward (:167-180)
  const double cost = S.ev_cost * rp;
  S.rew_ev = -(cost + p.ev_unserved_penalty * (unserved * unserved));
  R.common(cost, S.rew_ev, a, sc, bc, gc);            // :316-320
  R.put(6, power);
  R.put(7, unserved);
  R.put(8, (double)nact);
  R.put(9, (double)ndep);
  R.put(10, pv_cap - sc);
  R.put(11, es_cap - bc);
  R.put(12, grid_cap - gc);
}

// HSDevicesEnv.step (devices_env_hs.py:147-205).  Its draws on the resources
// are made on kwargs AFTER the meta it returns was copied (:158-160), so they
// never reach meta_state.
__device__ __forceinline__ void hs_devices(const pgw_hs_params& p, const pgw_hs_step_info& s, int rescale,
                                           bool reset, double a, const HSMeta& M, HSState& S, double& rp,
                                           double* ob, const HSRec& R) {
#pragma unroll
  for (int c = 0; c < PGW_HS_MAX_DEV; ++c) {
    if (c >= p.n_dev) break;
    ob[c] = rescale ? to_scaled(s.dev_obs[c], 0.0, p.dev_obs_high[c]) : s.dev_obs[c];
  }
  if (reset) return;
  if (rescale) {
    oob_note(p.oob, oob_bad(a));
    a = to_raw(a, p.dev_act_low, p.dev_act_high);
  }
  double sum = 0.0;
#pragma unroll
  for (int c = 0; c < PGW_HS_MAX_DEV; ++c) {
    if (c >= p.n_dev) break;
    sum = sum + s.dev_power[c];
  }
  rp = a * sum;
  double sc = 0.0, bc = 0.0, gc = 0.0;
  if (fabs(rp) < 0.0005) {                 // round(rp, 3) == 0.0
    S.dev_cost = 0.0;
  } else {
    sc = pymin(rp, M.pv);
    bc = pymin(M.es, rp - sc);
    gc = pymin(M.grid, rp - sc - bc);
    S.dev_cost = (0.0 * sc + s.grid_cost * gc + 0.0 * bc) / (sc + gc + bc);
  }
  const double cost = S.dev_cost * rp * p.dev_hours_per_step;
  S.rew_dev = -cost;
  R.common(cost, S.rew_dev, a, sc, bc, gc);           // :194-199
  R.put(6, rp);
  R.put(7, M.pv - sc);
  R.put(8, M.es - bc);
  R.put(9, M.grid - gc);
}

__global__ void __launch_bounds__(kBlock) k_hs(pgw_hs_params p_, pgw_hs_step_info s, int64_t n,
                                               pgw_hs_buffers b, const double* __restrict__ init_soc,
                                               int reset) {
  const pgw_hs_params& p = PGW_KERNARG0(pgw_hs_params);   // (no private copy)
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  HSMeta M;
  M.pv = b.pv_power_last ? b.pv_power_last[e] : 0.0;   // meta_state carried over (None = NaN)
  M.es = b.es_power_last[e];
  M.grid = p.max_grid_power;
  HSState S = {};
  S.soc = reset ? clip(init_soc[e], p.soc_min, p.soc_max) : b.soc[e];
  S.soc_cost = b.soc_cost[e];
  S.ev_cost = b.ev_cost[e];
  S.dev_cost = b.dev_cost[e];
  double rp_storage = 0.0;
  // The chain is unrolled over its (at most 4) slots and every case stores its
  // own observations: with a loop over n_comp the per-slot arrays (S.rp, ob)
  // were indexed dynamically and lived in scratch (288 B per lane).
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (c >= p.n_comp) break;
    const double a = reset ? 0.0 : ld(b.action, e, c);
    const HSRec R = {(!reset && b.step_meta) ? b.step_meta + (int64_t)c * PGW_HS_META_FIELDS * n : nullptr, n, e};
    double ob[8];
    const int off = p.obs_off[c];
    S.rp[c] = 0.0;
    switch (p.kind[c]) {
      case PGW_HS_PV:
        hs_pv(p, s, p.rescale[c], reset, a, p.pv_grid_aware ? b.min_voltage[e] : 0.0, M, S.rp[c], ob, R);
        st(b.obs, e, off, ob[0]);
        if (p.pv_grid_aware) st(b.obs, e, off + 1, ob[1]);
        break;
      case PGW_HS_STORAGE:
        if (!reset) hs_storage(p, s, p.rescale[c], a, M, S, S.rp[c], R);
        rp_storage = S.rp[c];
        ob[0] = S.soc;
        ob[1] = S.soc_cost;
        if (p.rescale[c]) {
          ob[0] = to_scaled(ob[0], p.soc_min, p.soc_max);
          ob[1] = to_scaled(ob[1], 0.0, p.max_storage_cost);
        }
        st(b.obs, e, off, ob[0]);
        st(b.obs, e, off + 1, ob[1]);
        break;
      case PGW_HS_EV:
        hs_ev(p, s, p.rescale[c], reset, a, n, e, b, M, S, S.rp[c], ob, R);
#pragma unroll
        for (int j = 0; j < 7; ++j) st(b.obs, e, off + j, ob[j]);
        break;
      default:
        hs_devices(p, s, p.rescale[c], reset, a, M, S, S.rp[c], ob, R);
#pragma unroll
        for (int j = 0; j < PGW_HS_MAX_DEV; ++j) {
          if (j >= p.n_dev) break;
          st(b.obs, e, off + j, ob[j]);
        }
        break;
    }
  }
  b.soc[e] = S.soc;
  b.soc_cost[e] = S.soc_cost;
  b.ev_cost[e] = S.ev_cost;
  b.dev_cost[e] = S.dev_cost;
  if (reset) return;
  // base_hs.py:157-180: real power and the house reward, components in chain order
  double rp = 0.0, rew = 0.0;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (c >= p.n_comp) break;
    rp = rp + S.rp[c];
    const int k = p.kind[c];
    const double r = k == PGW_HS_PV ? 0.0
                   : k == PGW_HS_STORAGE ? hs_storage_reward(p, M, S, rp_storage)
                   : k == PGW_HS_EV ? S.rew_ev : S.rew_dev;
    rew = rew + r;
  }
  b.real_power[e] = rp;
  b.reward[e] = rew;
  b.es_power_last[e] = M.es;
  if (b.pv_power_last) b.pv_power_last[e] = M.pv;
  if (b.meta_out) {
    b.meta_out[e] = M.pv;
    b.meta_out[n + e] = M.es;
    b.meta_out[2 * n + e] = M.grid;
  }
}

static int32_t hs_check(const pgw_hs_params* p, const pgw_hs_step_info* s, int64_t n, const pgw_hs_buffers& b) {
  PGW_REQUIRE(p && s && n >= 0, "pgw_hs: null argument");
  PGW_REQUIRE(p->n_comp >= 1 && p->n_comp <= 4, "pgw_hs: bad n_comp");
  PGW_REQUIRE(p->n_veh >= 0 && p->n_veh <= PGW_HS_MAX_VEHICLES, "pgw_hs: bad n_veh");
  PGW_REQUIRE(p->n_dev >= 0 && p->n_dev <= PGW_HS_MAX_DEV, "pgw_hs: bad n_dev");
  int seen = 0;
  for (int c = 0; c < p->n_comp; ++c) {
    PGW_REQUIRE(p->kind[c] >= 0 && p->kind[c] <= 3 && !(seen & (1 << p->kind[c])),
                "pgw_hs: component kinds must be distinct PGW_HS_* values");
    seen |= 1 << p->kind[c];
  }
  PGW_REQUIRE(b.obs.ptr && b.soc && b.soc_cost && b.ev_cost && b.dev_cost && b.es_power_last,
              "pgw_hs: null buffer");
  PGW_REQUIRE(!(seen & (1 << PGW_HS_EV)) || (b.ev_req && b.ev_charging), "pgw_hs: null EV buffer");
  PGW_REQUIRE(!p->pv_grid_aware || ((seen & (1 << PGW_HS_PV)) && b.min_voltage),
              "pgw_hs: the grid-aware PV needs min_voltage");
  return PGW_OK;
}

}  // namespace pgw

using namespace pgw;

extern "C" {

int32_t pgw_hs_reset(const pgw_hs_params* p, const pgw_hs_step_info* s, int64_t n, const double* init_soc,
                     pgw_hs_buffers b, void* stream) {
  int32_t rc = hs_check(p, s, n, b);
  if (rc) return rc;
  PGW_REQUIRE(init_soc, "pgw_hs_reset: null init_soc");
  if (n == 0) return PGW_OK;
  hipLaunchKernelGGL(k_hs, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, *p, *s, n, b, init_soc, 1);
  return check_launch("k_hs(reset)");
}

int32_t pgw_hs_step(const pgw_hs_params* p, const pgw_hs_step_info* s, int64_t n, pgw_hs_buffers b,
                    void* stream) {
  int32_t rc = hs_check(p, s, n, b);
  if (rc) return rc;
  PGW_REQUIRE(b.action.ptr && b.reward && b.real_power, "pgw_hs_step: null buffer");
  if (n == 0) return PGW_OK;
  hipLaunchKernelGGL(k_hs, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, *p, *s, n, b,
                     (const double*)nullptr, 0);
  return check_launch("k_hs(step)");
}

}  // extern "C"
