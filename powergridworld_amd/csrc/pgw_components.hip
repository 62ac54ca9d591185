// Component step kernels: battery, PV, building, EV, multi-component reduce.
// One thread per env; env-minor SoA state, so every per-env load/store of a
// field is a contiguous, fully coalesced 512-B wave access.
#include <cstdarg>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <type_traits>

#include "pgw_common.h"

namespace pgw {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int32_t check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return PGW_ERR_HIP;
  }
  return PGW_OK;
}

// ====================================================================== battery
// S = double (pgw_mat) or float (pgw_matf, the _f32 entries: fp32 storage,
// fp64 arithmetic).
template <class S, class Mt>
__global__ void __launch_bounds__(kBlock) k_battery_reset(pgw_battery_params p, int64_t n,
                                                          const S* __restrict__ init,
                                                          S* __restrict__ soc, Mt obs) {
  int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  // a given init_storage is clipped (energy_storage_env.py:86-95), a drawn one
  // (truncnorm * std + mean, :80-84) is not
  double s = p.sampled_init ? (double)init[e] : clip((double)init[e], p.soc_min, p.soc_max);
  soc[e] = (S)s;
  st(obs, e, 0, battery_obs(p, s));
}

// One env's EnergyStorageEnv.step; returns its real power (-power, :150).
template <class S, class Mt>
__device__ __forceinline__ double battery_step_env(const pgw_battery_params& p, int64_t e, const Mt& act,
                                                   S* __restrict__ soc, const Mt& obs) {
  double s = soc[e];
  double power = battery_step(p, ld(act, e, 0), s);
  soc[e] = (S)s;
  st(obs, e, 0, battery_obs(p, s));
  return -power;
}

template <class S, class Mt>
__global__ void __launch_bounds__(kBlock) k_battery_step(pgw_battery_params p, int64_t n,
                                                         Mt act, S* __restrict__ soc,
                                                         Mt obs, S* __restrict__ rp) {
  int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  rp[e] = (S)battery_step_env(p, e, act, soc, obs);
}

// ====================================================================== PV
// One env's PVEnv obs (+ step when act.ptr): obs first (pre-advance, :143).
// Mt = pgw_mat or pgw_matf (the _f32 entries: fp32 storage, fp64 arithmetic).
template <class Mt>
__device__ __forceinline__ double pv_step_env(const pgw_pv_params& p, int64_t e, double pmax, const Mt& act,
                                              const double* __restrict__ vmin, const Mt& obs) {
  st(obs, e, 0, pv_obs(p, pmax));
  if (p.grid_aware) {
    double v = vmin[e];
    st(obs, e, 1, p.rescale ? to_scaled(v, p.vmin_low, p.vmin_high) : v);
  }
  return act.ptr ? pv_real_power(p, ld(act, e, 0), pmax) : 0.0;
}

template <class S, class Mt>
__global__ void __launch_bounds__(kBlock) k_pv(pgw_pv_params p, int64_t n, double pmax, Mt act,
                                               const double* __restrict__ vmin, Mt obs,
                                               S* __restrict__ rp) {
  int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  const double r = pv_step_env(p, e, pmax, act, vmin, obs);
  if (rp) rp[e] = (S)r;
}

// Debug phase trace (pgw_debug_mc_trace): the TR instantiations of k_mc_step
// and k_ma_step have lane 0 of every wave record wall_clock64() (100 MHz) at
// its phase boundaries into g_mc_trace[(block * 8 + wave) * 8 + slot]; the
// product launches the TR = false kernels, which hold no trace code at all.
// Slots: 0 entry, 1 after the block's staging barrier, 2 the wave's component
// (or walk group) done, 3 the building's loads arrived, 4 the EV fold and
// finish done, 5 after the final barrier, 6 the sums written, 7 the building's
// state update and reward done (its obs next).  16 waves per block.
__device__ long long* g_mc_trace = nullptr;
template <bool TR>
__device__ __forceinline__ void mc_trace(long long* tr, int slot) {
  if constexpr (TR) {
    if ((threadIdx.x & 63) == 0) {
      typedef __attribute__((address_space(1))) long long* gptr;
      ((gptr)tr)[((int64_t)blockIdx.x * 16 + (threadIdx.x >> 6)) * 8 + slot] = wall_clock64();
    }
  }
}

// A component's real power and reward as stored (S-rounded), handed to the
// block's sums in registers: reading the component's own stores back cost a
// store-to-load round trip at the end of every component wave.
struct RpRew {
  double rp, rew;
};

// ====================================================================== building
template <class S, class Mt>
__global__ void __launch_bounds__(kBlock) k_building_reset(pgw_building_params p, pgw_building_exo ex0,
                                                           int64_t n, S* __restrict__ x,
                                                           S* __restrict__ pcons,
                                                           S* __restrict__ rstate,
                                                           pgw_building_ext ext, Mt obs) {
  int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  double xs[5], T[5];
#pragma unroll
  for (int z = 0; z < 5; ++z) {
    xs[z] = x[z * n + e];
    T[z] = p.T_init[z];
  }
  // two filter updates with the same u (five_zone_rom_env.py:160-173)
  for (int it = 0; it < 2; ++it) {
    building_state_update(p, ex0, T, nullptr, xs);
#pragma unroll
    for (int z = 0; z < 5; ++z) {
      double yhat = p.C[z] * xs[z];
      double yact = T[z] - p.mean[z];
      xs[z] = xs[z] + p.K[z] * (yact - yhat);
    }
  }
#pragma unroll
  for (int z = 0; z < 5; ++z) {
    x[z * n + e] = (S)xs[z];
    T[z] = p.C[z] * xs[z] + p.mean[z];               // temp_dynamics (dynamics.py:75-85)
  }
  pcons[e] = (S)0.0;
  BuildingExt xv = building_ext(ext, e);
  building_write_obs(p, T, ex0, 0.0, xv, [&](int j, double v) { st(obs, e, j, v); });
  if (rstate) rstate[e] = (S)building_reward(p, T, ex0.comfort_lb, ex0.comfort_ub, 0.0);
}

// The fused kernels' building wave reads its parameters (pgw_building_params,
// BldDerived: ~1.6 KB) from LDS: from the kernel-argument segment they are ~30
// dependent scalar loads, each waited for before its use (the SGPRs cannot hold
// them all), and the phase trace put the step at 8.6 us, 4.5 of them the obs
// loop (tools/gpu/mc_trace.py).  The wave copies them itself -- its 64 lanes
// issue the copy together with the step's own HBM loads, one round trip for
// both -- so no block barrier is involved.
__device__ __forceinline__ void bld_stage_wave(const pgw_building_params& p, const BldDerived& d,
                                               pgw_building_params& sp, BldDerived& sd, int lane) {
  constexpr int kP = (int)(sizeof(pgw_building_params) / 8), kD = (int)(sizeof(BldDerived) / 8);
  static_assert(sizeof(pgw_building_params) % 8 == 0 && sizeof(BldDerived) % 8 == 0, "staged as doubles");
  double v[(kP + kD + 63) / 64];
#pragma unroll
  for (int k = 0; k < (kP + kD + 63) / 64; ++k) {
    const int i = lane + 64 * k;
    v[k] = i < kP ? reinterpret_cast<const double*>(&p)[i]
                  : i < kP + kD ? reinterpret_cast<const double*>(&d)[i - kP] : 0.0;
  }
#pragma unroll
  for (int k = 0; k < (kP + kD + 63) / 64; ++k) {
    const int i = lane + 64 * k;
    if (i < kP) reinterpret_cast<double*>(&sp)[i] = v[k];
    else if (i < kP + kD) reinterpret_cast<double*>(&sd)[i - kP] = v[k];
  }
  // (one wave: its LDS operations complete in order; the fence keeps the
  // compiler from moving the other lanes' reads above these writes)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// The std building step in two parts: its per-env inputs (the 6 actions, x_k)
// and the step from them, so that the fused kernels' building wave can issue
// the inputs' HBM loads together with its parameter staging (bld_stage_wave).
struct BldIn {
  double av[6], xs[5];
};
template <class S, class Mt>
__device__ __forceinline__ void bld_std_load(int64_t n, int64_t e, const Mt& act, const S* __restrict__ x,
                                             BldIn& in) {
#pragma unroll
  for (int j = 0; j < 6; ++j) in.av[j] = ld(act, e, j);
#pragma unroll
  for (int z = 0; z < 5; ++z) in.xs[z] = x[z * n + e];
}
template <class S, class Mt, bool TR = false>
__device__ __forceinline__ double bld_std_from(const pgw_building_params& p, const BldDerived& d,
                                               const pgw_building_exo& ex, const pgw_building_exo& exn,
                                               int64_t n, int64_t e, BldIn& in, S* __restrict__ x,
                                               S* __restrict__ pcons, S* __restrict__ rout,
                                               S* __restrict__ rstate, int32_t lagged, const Mt& obs,
                                               double* fresh_out) {
  double fresh;
  long long* const tr = TR ? g_mc_trace : nullptr;
  const double pc = bld_std_step(p, d, ex, exn, in.av, in.xs, fresh, [&](int j, double v) { st(obs, e, j, v); },
                                 [&](int slot) { mc_trace<TR>(tr, slot); });
#pragma unroll
  for (int z = 0; z < 5; ++z) x[z * n + e] = (S)in.xs[z];
  pcons[e] = (S)pc;
  if (rout) rout[e] = lagged ? rstate[e] : (S)fresh;
  if (rstate) rstate[e] = (S)fresh;
  if (fresh_out) *fresh_out = (double)(S)fresh;
  return pc;
}

// The fused kernels' std building wave (all its lanes, e < n or not: every
// lane copies its share of the parameters): inputs and parameter copy in one
// round trip, then the step from LDS.  Returns the stored (p_consumed, reward).
template <class S, class Mt, bool TR>
__device__ __forceinline__ RpRew bld_wave_std(const pgw_building_params& p, const BldDerived& d,
                                              pgw_building_params& sp, BldDerived& sd,
                                              const pgw_building_exo& ex, const pgw_building_exo& exn,
                                              int64_t n, int64_t e, const Mt& act, S* __restrict__ x,
                                              S* __restrict__ pcons, S* __restrict__ rstate, const Mt& obs) {
  BldIn in;
  if (e < n) bld_std_load(n, e, act, x, in);
  bld_stage_wave(p, d, sp, sd, (int)(threadIdx.x & 63));
  RpRew r{0.0, 0.0};
  if (e < n) {
    double fresh = 0.0;
    const S pc = (S)bld_std_from<S, Mt, TR>(sp, sd, ex, exn, n, e, in, x, pcons, (S*)nullptr, rstate, 0, obs,
                                            &fresh);
    r = {(double)pc, fresh};
  }
  return r;
}

// One env's FiveZoneROMEnv.step_ (:183-225); returns p_consumed (its real power).
// STD: the reference's default model/obs layout (bld_is_std), via bld_std_step.
template <bool STD, class S = double, class Mt = pgw_mat, bool TR = false>
__device__ __forceinline__ double building_step_env(const pgw_building_params& p, const BldDerived& d,
                                                    const pgw_building_exo& ex,
                                                    const pgw_building_exo& exn, int64_t n, int64_t e,
                                                    const Mt& act, S* __restrict__ x,
                                                    S* __restrict__ pcons, S* __restrict__ rout,
                                                    S* __restrict__ rstate, int32_t lagged,
                                                    const pgw_building_ext& ext, const Mt& obs,
                                                    double* fresh_out = nullptr) {
  if constexpr (STD) {
    BldIn in;
    bld_std_load(n, e, act, x, in);
    return bld_std_from<S, Mt, TR>(p, d, ex, exn, n, e, in, x, pcons, rout, rstate, lagged, obs, fresh_out);
  }
  double a[6], xs[5], T[5];
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double v = ld(act, e, j);
    bad = bad || oob_bad(v);
    a[j] = p.rescale ? to_raw(v, p.act_low[j], p.act_high[j]) : v;
  }
  if (p.rescale) oob_note(p.oob, bad);
#pragma unroll
  for (int z = 0; z < 5; ++z) {
    xs[z] = x[z * n + e];
    T[z] = p.C[z] * xs[z] + p.mean[z];   // zone temps are a pure function of x_k
  }
  building_state_update(p, ex, T, a, xs);
#pragma unroll
  for (int z = 0; z < 5; ++z) {
    x[z * n + e] = (S)xs[z];
    T[z] = p.C[z] * xs[z] + p.mean[z];
  }
  double pc = building_p_consumed(a, ex.T_oa);
  pcons[e] = (S)pc;
  double fresh = building_reward(p, T, exn.comfort_lb, exn.comfort_ub, pc);
  if (rout) rout[e] = lagged ? rstate[e] : (S)fresh;
  if (rstate) rstate[e] = (S)fresh;
  if (fresh_out) *fresh_out = (double)(S)fresh;
  BuildingExt xv = building_ext(ext, e);
  building_write_obs(p, T, exn, pc, xv, [&](int j, double v) { st(obs, e, j, v); });
  return pc;
}

template <bool STD, class S, class Mt>
__global__ void __launch_bounds__(kBlock) k_building_step(pgw_building_params p_, BldDerived d,
                                                          pgw_building_exo ex,
                                                          pgw_building_exo exn, int64_t n, Mt act,
                                                          S* __restrict__ x,
                                                          S* __restrict__ pcons,
                                                          S* __restrict__ rout,
                                                          S* __restrict__ rstate, int32_t lagged,
                                                          pgw_building_ext ext, Mt obs) {
  const pgw_building_params& p = PGW_KERNARG0(pgw_building_params);   // (no private copy)
  int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  (void)building_step_env<STD, S, Mt>(p, d, ex, exn, n, e, act, x, pcons, rout, rstate, lagged, ext, obs);
}

// ====================================================================== EV
template <class S>
__global__ void __launch_bounds__(kBlock) k_ev_reset(int64_t n, int32_t V, int32_t W,
                                                     const double* __restrict__ req0,
                                                     S* __restrict__ req,
                                                     uint64_t* __restrict__ chg) {
  int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  for (int v = 0; v < V; ++v) req[(int64_t)v * n + e] = (S)req0[v];
  for (int w = 0; w < W; ++w) chg[(int64_t)w * n + e] = 0ull;
}

// randomize=True (ev_charging_env.py:154-156): every env restores its own
// sampled vehicles' requirements.
template <class S>
__global__ void __launch_bounds__(kBlock) k_ev_reset_tables(int64_t n, int32_t V, int32_t W,
                                                            const double* __restrict__ req0,
                                                            S* __restrict__ req,
                                                            uint64_t* __restrict__ chg) {
  int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  for (int v = 0; v < V; ++v) req[(int64_t)v * n + e] = (S)req0[(int64_t)v * n + e];
  for (int w = 0; w < W; ++w) chg[(int64_t)w * n + e] = 0ull;
}

// ev_charging_env.py:171-264.  Vehicles are visited in ascending index order
// (the reference iterates a Python set of small ints); only vehicles parked now
// or at the previous step can contribute (`scan`, uniform across the wave).
// One env's EVChargingEnv.step (:171-264); writes rp[e] and rew[e].
// MODE (uniform, chosen once per call by ev_step_env): 0 = the host's
// time-left table with reciprocals (exact_div), 1 = randomize's per-env tables,
// 2 = time left divided in the kernel.  Instantiated per mode so the vehicle
// loop carries no per-vehicle branch and no unused IEEE division.
enum { kEvTable = 0, kEvPerEnv = 1, kEvDivide = 2 };
// The vehicle walk's sums (demand, energy consumed, deficit sum, unserved) run
// in kEvGroups groups of consecutive chunks: group g covers chunks [g K, g K + K)
// of the step's scan, K = ceil(chunks / kEvGroups), each group summed from 0 in
// vehicle order, the totals ((0 + p0) + p1) + p2 + p3.  One lane walking every
// chunk folds at the group boundaries; k_mc_step's split EV waves (one group
// each, below) fold the same partials after a block barrier -- so both forms are
// bit-identical, whichever kernel steps the env.  (The reference sums demand,
// consumed and unserved with sequential `+=` in the charging set's iteration
// order, ev_charging_env.py:204-242; only the mean deficit is np.mean, :252,
// pairwise from 8 elements on.  With more than one group the totals here are
// ((p0 + p1) + p2) + p3 instead, a rounding difference of an ulp or so: the
// goldens compare at rtol 1e-12, the north star allows 1e-6.)
// A lane's double, read by the whole wave from lane l (uniform): two
// v_readlane_b32 into SGPRs.
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long x = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(x & 0xffffffffll), l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(x >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// The host's time-left table is read by readlane (ev_walk), which needs every
// lane of the wave walking; the grid's last, partial wave divides in the
// kernel instead (kEvDivide: (end_park - t) / 60 and r / tl with the same IEEE
// operations as the host table and exact_div -- the same values).
__device__ __forceinline__ bool ev_table_ok(const pgw_ev_step_info& s) {
  return s.tl_rcp != nullptr && __builtin_amdgcn_read_exec() == ~0ull;
}
constexpr int kEvChunk = 8;
constexpr int kEvGroups = 8;
struct EvSums {
  double demand, consumed, dsum, unserved;
  int dcnt, nact;
};
__device__ __forceinline__ int ev_chunks(const pgw_ev_step_info& s) {       // uniform
  int c = 0;
  for (int w = 0; w < s.n_words; ++w) c += (__builtin_popcountll(s.scan[w]) + kEvChunk - 1) / kEvChunk;
  return c;
}
__device__ __forceinline__ int ev_group_len(int chunks) { return max(1, (chunks + kEvGroups - 1) / kEvGroups); }
// The one-lane walk's folded totals wait in LDS (indexed by thread; blocks are
// at most 512 threads): four more doubles held in registers through the walk
// took the EV kernels from 3 to 2 waves per SIMD.
constexpr int kEvFoldThreads = 512;
// every block that runs the one-lane walk must fit: k_ev_step (kBlock), k_mc_step
// unsplit (64 x 4 components; its split blocks walk with SPLIT = true, no fold
// buffer), k_ma_step (64 x slots)
static_assert(kBlock <= kEvFoldThreads, "s_ev_fold: k_ev_step block");
static_assert(64 * 4 <= kEvFoldThreads, "s_ev_fold: k_mc_step block");
static_assert(64 * PGW_MA_MAX_SLOTS <= kEvFoldThreads, "s_ev_fold: k_ma_step block");
__shared__ double s_ev_fold[4][kEvFoldThreads];

// The env's EV action (:176-181): loaded at the top, used only once the walk's
// first loads are out -- the charge energy in each chunk's processing
// (ev_kwh_of), the out-of-bounds note after the walk (ev_note, once per env:
// only one of the split waves notes it).  A branch on the action before the
// walk (the note's atomic) made the vehicle loads wait for its round trip.
template <class Mt>
__device__ __forceinline__ double ev_act(const pgw_ev_step_info& s, int64_t e, const Mt& act) {
  return act.ptr ? ld(act, e, 0) : s.action_default;
}
// The env's charge energy this step (:215-223)
__device__ __forceinline__ double ev_kwh_of(const pgw_ev_params& p, double a) {
  if (p.rescale) a = to_raw(a, 0.0, 1.0);
  return a * p.rate * p.hours_per_step;
}
__device__ __forceinline__ void ev_note(const pgw_ev_params& p, double a) {
  if (p.rescale) oob_note(p.oob, oob_bad(a));
}

// Walks chunks [c_lo, c_hi) of the scan (:224-252).  SPLIT = false: the whole
// scan in one lane, folding at the group boundaries, the charging bits stored
// per word.  SPLIT = true: one group's chunks; the bits are ORed into the
// block's s_bits[word][lane] and the group's partial sums returned unfolded.
template <int MODE, bool SPLIT, class S, bool TR = false>
__device__ __forceinline__ EvSums ev_walk(const pgw_ev_params& p, const pgw_ev_step_info& s, int64_t n,
                                          int64_t e, double act_raw, const double* __restrict__ endp,
                                          S* __restrict__ req, uint64_t* __restrict__ chg, int c_lo,
                                          int c_hi, int K, uint64_t* s_bits, int lane) {
  double demand = 0.0, consumed = 0.0, dsum = 0.0, unserved = 0.0;   // the current group's
  int dcnt = 0, nact = 0;
  int ctr = 0, next_fold = K;                        // uniform chunk counter
  bool folded = false;                               // (uniform) s_ev_fold holds a total
  const int tid = threadIdx.x;
  // The scan mask is wave-uniform (scalar), so the vehicle loop is too.  The
  // vehicles go in chunks of kEvChunk: the chunk's requirements are loaded back
  // to back (one memory round trip per chunk, not per vehicle); then every
  // vehicle's quantities (deficit, charge, the new requirement) are computed
  // with no branch -- independent chains the scheduler interleaves, where one
  // vehicle at a time was a single dependent chain per wave (~0.2 us per
  // vehicle at one wave per SIMD) -- and last the sums run over the chunk in
  // ascending vehicle order, by selects, exactly as one vehicle at a time.
  // Both passes walk the same chunk mask, so no index array is needed.
  struct Chunk {
    uint64_t bits;
    double rs[kEvChunk], tls[kEvChunk], rcs[kEvChunk];
    bool wins[kEvChunk];
  };
  auto take = [](uint64_t& scan) {                   // the next <= kEvChunk vehicle bits
    uint64_t c = scan;
#pragma unroll
    for (int i = 0; i < kEvChunk; ++i) scan &= scan - 1;
    return c & ~scan;
  };
  for (int w = 0; w < s.n_words; ++w) {
    uint64_t scan = s.scan[w];
    const int base = ctr, nc = (__builtin_popcountll(scan) + kEvChunk - 1) / kEvChunk;
    ctr += nc;
    const int lo = max(base, c_lo), hi = min(base + nc, c_hi);
    if (SPLIT && lo >= hi) continue;                 // (uniform) none of this group's chunks
    for (int i = base; i < lo; ++i) (void)take(scan);
    int budget = hi - lo, at = lo;
    auto take_mine = [&]() -> uint64_t { return budget-- > 0 ? take(scan) : 0ull; };
    const uint64_t win = s.window[w];
    const uint64_t prev = chg[(int64_t)w * n + e];
    uint64_t now_bits = 0ull;
    // kEvTable: the word's 64 table entries, one per lane (a coalesced 1 KB
    // load with the first chunks' requirements); vehicle b's pair is then
    // read from lane b (readlane, no memory operation), where a 16-byte
    // broadcast load per vehicle doubled the chunk's memory instructions and
    // held 4 VGPRs per vehicle in flight.  Only in a whole wave (ev_table_ok):
    // the callers run the walk for their e < n lanes, and a lane that is off
    // never loads its entry.
    double lane_tl = 0.0, lane_rc = 0.0;
    if constexpr (MODE == kEvTable) {
      const int vl = w * 64 + (int)(threadIdx.x & 63);
      if (vl < p.n_vehicles) {
        const double2 q = reinterpret_cast<const double2*>(s.tl_rcp)[vl];
        lane_tl = q.x;
        lane_rc = q.y;
      }
    }
    // the chunk's loads all go out before any is used: the requirements
    // (vector) and the vehicles' time left (uniform: scalar loads)
    auto load = [&](Chunk& C) {
      uint64_t m = C.bits;
#pragma unroll
      for (int i = 0; i < kEvChunk; ++i) {
        const int b = m ? __builtin_ctzll(m) : 0;    // past the chunk's end: a harmless reload
        const int v = w * 64 + b;
        C.rs[i] = (double)req[(int64_t)v * n + e];
        if constexpr (MODE == kEvPerEnv) {       // randomize: this env's own vehicle table
          const double en = s.env_endp[(int64_t)v * n + e];
          C.tls[i] = (en - s.time) / 60.0;
          C.rcs[i] = 0.0;
          C.wins[i] = (s.time >= s.env_start[(int64_t)v * n + e]) && (s.time <= floor(en));
        } else if constexpr (MODE == kEvTable) { // host table: read at use (process), from its lane
          C.tls[i] = 0.0;
          C.rcs[i] = 0.0;
        } else {
          C.tls[i] = (endp[v] - s.time) / 60.0;
          C.rcs[i] = 0.0;
        }
        if constexpr (MODE != kEvPerEnv) C.wins[i] = (win >> b) & 1ull;
        m &= m - 1;
      }
    };
    // the chunk's new requirements go out after the pair is processed
    // (store_nr): a store between the pair's two chunks made the second one
    // wait for it (vmcnt counts loads and stores in order)
    auto store_nr = [&](const Chunk& C, const S (&val)[kEvChunk]) {
      uint64_t m = C.bits;
#pragma unroll
      for (int i = 0; i < kEvChunk; ++i) {
        const bool in = m != 0;
        const int b = in ? __builtin_ctzll(m) : 0;
        m &= m - 1;
        if (in) req[(int64_t)(w * 64 + b) * n + e] = val[i];
      }
    };
    auto process = [&](const Chunk& C, S (&val)[kEvChunk]) {
      if (!SPLIT && at == next_fold) {               // (uniform) a group boundary
        // (the first total is the first group's sum: 0.0 + p0 == p0, a sum from
        // +0.0 being never -0.0)
        const double q[4] = {demand, consumed, dsum, unserved};
#pragma unroll
        for (int j = 0; j < 4; ++j) s_ev_fold[j][tid] = folded ? s_ev_fold[j][tid] + q[j] : q[j];
        folded = true;
        demand = consumed = dsum = unserved = 0.0;
        next_fold += K;
      }
      ++at;
      const double kwh = ev_kwh_of(p, act_raw);      // (after the chunk's loads issued)
      double df[kEvChunk], cv[kEvChunk];
      bool act[kEvChunk], chg_now[kEvChunk], dep[kEvChunk];
      uint64_t m = C.bits;
#pragma unroll
      for (int i = 0; i < kEvChunk; ++i) {
        const bool in = m != 0;                      // uniform: the chunk's tail is not
        const int b = in ? __builtin_ctzll(m) : 0;
        m &= m - 1;
        const double r = C.rs[i];
        double tl = C.tls[i], rc = C.rcs[i];
        if constexpr (MODE == kEvTable) {
          tl = readlane_f64(lane_tl, b);
          rc = readlane_f64(lane_rc, b);
        }
        act[i] = in && C.wins[i] && (r > 0.0);
        chg_now[i] = act[i] && (tl > 0.0);
        dep[i] = in && !act[i] && ((prev >> b) & 1ull);   // departed: not charging now (:239-243)
        if constexpr (MODE == kEvTable) df[i] = pymax(0.0, p.rate - exact_div(r, tl, rc));
        else df[i] = pymax(0.0, p.rate - r / tl);
        cv[i] = pymin(kwh, r);
        // unconditional (the unchanged value where not charging): a store
        // under a branch leaves the compiler no static count of outstanding
        // memory operations, and it then waits for all of them (vmcnt(0)),
        // stores included, before every later load's use
        val[i] = (S)(chg_now[i] ? r - cv[i] : r);
      }
      m = C.bits;
#pragma unroll
      for (int i = 0; i < kEvChunk; ++i) {
        const uint64_t lo_bit = m & (0ull - m);      // the chunk's i-th vehicle bit (0 past its end)
        m &= m - 1;
        demand = act[i] ? demand + C.rs[i] : demand;
        nact += act[i] ? 1 : 0;
        now_bits |= act[i] ? lo_bit : 0ull;
        dsum = chg_now[i] ? dsum + df[i] : dsum;
        consumed = chg_now[i] ? consumed + cv[i] : consumed;
        dcnt += chg_now[i] ? 1 : 0;
        unserved = dep[i] ? unserved + C.rs[i] : unserved;
      }
    };
    // chunks in pairs: both chunks' loads go out before either is processed
    // (unconditionally: an empty second chunk reloads vehicle w*64, harmless),
    // then the two are processed in order -- one memory round trip per pair.
    // (A rotating two-buffer pipeline, the next pair's loads before this
    // pair's processing, compiled to one round trip per chunk: the
    // per-wave phase trace showed each chunk costing a full round trip.)
    // (randomize's per-env tables load two more values per vehicle: one chunk
    // at a time there, pairs spilled)
    bool first_pair = true;                          // (debug trace only)
    while (budget > 0) {                             // (uniform)
      Chunk A, B;
      S va[kEvChunk], vb[kEvChunk];
      A.bits = take_mine();
      load(A);
      if constexpr (MODE != kEvPerEnv) {
        B.bits = take_mine();
        load(B);
      }
      process(A, va);
      if constexpr (TR) { if (demand != -1.0 && first_pair) mc_trace<TR>(g_mc_trace, 3); }
      if constexpr (MODE != kEvPerEnv)
        if (B.bits) process(B, vb);
      if constexpr (TR) { if (demand != -1.0 && first_pair) mc_trace<TR>(g_mc_trace, 7); }
      first_pair = false;
      store_nr(A, va);
      if constexpr (MODE != kEvPerEnv)
        if (B.bits) store_nr(B, vb);
    }
    if constexpr (SPLIT) {
      if (now_bits) atomicOr(reinterpret_cast<unsigned long long*>(&s_bits[w * 64 + lane]),
                             (unsigned long long)now_bits);
    } else {
      chg[(int64_t)w * n + e] = now_bits;
    }
  }
  EvSums t{demand, consumed, dsum, unserved, 0, 0};
  if (!SPLIT && folded) {
    t.demand = s_ev_fold[0][tid] + demand;
    t.consumed = s_ev_fold[1][tid] + consumed;
    t.dsum = s_ev_fold[2][tid] + dsum;
    t.unserved = s_ev_fold[3][tid] + unserved;
  }
  t.dcnt = dcnt;
  t.nact = nact;
  return t;
}

// The step's state, reward and obs from the walk's totals (:253-262, :135-142).
template <class S, class Mt>
__device__ __forceinline__ RpRew ev_finish(const pgw_ev_params& p, const pgw_ev_step_info& s, int64_t e,
                                          const EvSums& t, const Mt& obs, S* __restrict__ rp,
                                          S* __restrict__ rew) {
  double st_[6];
  st_[0] = s.next_time;
  st_[1] = p.mult * (double)t.nact;
  st_[2] = p.mult * t.consumed;
  st_[3] = p.mult * t.demand;
  st_[4] = t.dcnt ? t.dsum / (double)t.dcnt : 0.0;
  st_[5] = t.unserved;
  const S rp_e = (S)(p.mult * t.consumed);           // :255
  rp[e] = rp_e;
  // step_reward :135-142
  double ur = -p.u_pen * (st_[5] * st_[5]);
  double pk = pymax(0.0, st_[2] - p.thr);
  double pr = -p.p_pen * (pk * pk);
  const S rew_e = (S)((ur + pr) / p.reward_scale);
  rew[e] = rew_e;
#pragma unroll
  for (int j = 0; j < 6; ++j)
    st(obs, e, j, p.rescale ? to_scaled(st_[j], p.obs_low[j], p.obs_high[j]) : st_[j]);
  return {(double)rp_e, (double)rew_e};
}

template <int MODE, class S, class Mt>
__device__ __forceinline__ RpRew ev_step_mode(const pgw_ev_params& p, const pgw_ev_step_info& s, int64_t n,
                                             int64_t e, const Mt& act, const double* __restrict__ endp,
                                             S* __restrict__ req, uint64_t* __restrict__ chg,
                                             const Mt& obs, S* __restrict__ rp,
                                             S* __restrict__ rew) {
  const double a = ev_act(s, e, act);
  const int nc = ev_chunks(s);
  const EvSums t = ev_walk<MODE, false>(p, s, n, e, a, endp, req, chg, 0, nc, ev_group_len(nc), nullptr, 0);
  ev_note(p, a);
  return ev_finish(p, s, e, t, obs, rp, rew);
}

template <class S, class Mt>
__device__ __forceinline__ RpRew ev_step_env(const pgw_ev_params& p, const pgw_ev_step_info& s, int64_t n,
                                            int64_t e, const Mt& act, const double* __restrict__ endp,
                                            S* __restrict__ req, uint64_t* __restrict__ chg,
                                            const Mt& obs, S* __restrict__ rp,
                                            S* __restrict__ rew) {
  if (s.env_start) return ev_step_mode<kEvPerEnv>(p, s, n, e, act, endp, req, chg, obs, rp, rew);
  if (ev_table_ok(s)) return ev_step_mode<kEvTable>(p, s, n, e, act, endp, req, chg, obs, rp, rew);
  return ev_step_mode<kEvDivide>(p, s, n, e, act, endp, req, chg, obs, rp, rew);
}

// Group g's part of the walk (k_mc_step's split EV waves).
template <class S, class Mt, bool TR = false>
__device__ __forceinline__ EvSums ev_step_group(const pgw_ev_params& p, const pgw_ev_step_info& s, int64_t n,
                                                int64_t e, const Mt& act, const double* __restrict__ endp,
                                                S* __restrict__ req, uint64_t* __restrict__ chg, int g,
                                                uint64_t* s_bits, int lane) {
  const double a = ev_act(s, e, act);
  const int nc = ev_chunks(s), K = ev_group_len(nc);
  const int lo = min(g * K, nc), hi = min(lo + K, nc);
  EvSums t;
  if (s.env_start) t = ev_walk<kEvPerEnv, true>(p, s, n, e, a, endp, req, chg, lo, hi, K, s_bits, lane);
  else if (ev_table_ok(s)) t = ev_walk<kEvTable, true, S, TR>(p, s, n, e, a, endp, req, chg, lo, hi, K, s_bits, lane);
  else t = ev_walk<kEvDivide, true>(p, s, n, e, a, endp, req, chg, lo, hi, K, s_bits, lane);
  if (g == 0) ev_note(p, a);
  return t;
}

template <class S, class Mt>
__global__ void __launch_bounds__(kBlock) k_ev_step(pgw_ev_params p, pgw_ev_step_info s, int64_t n,
                                                    Mt act, const double* __restrict__ endp,
                                                    S* __restrict__ req,
                                                    uint64_t* __restrict__ chg, Mt obs,
                                                    S* __restrict__ rp,
                                                    S* __restrict__ rew) {
  int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  (void)ev_step_env(p, s, n, e, act, endp, req, chg, obs, rp, rew);
}

// ---- lanes over vehicles (env-major requirements) --------------------------
// req[e * VP + v], VP = LPE * W: an env's vehicles are one contiguous row, and
// LPE lanes (16, 32 or 64: the smallest power of two >= V up to 64) serve one
// env, lane j its vehicles j, j + 64, ... (word w: vehicle w * 64 + j).  A
// wave loads EPW = 64 / LPE env rows per instruction, coalesced, and runs
// NP env passes with every pass's loads out before any is used: one memory
// round trip per wave.  Sums: per lane over its words in order from 0, then a
// butterfly over the env's lanes, partners at distance LPE/2 first (every lane
// ends with the same value); counts and the charging bits from ballots.
template <int LPE>
__device__ __forceinline__ double ev_lanes_sum(double x) {
#pragma unroll
  for (int m = LPE / 2; m >= 1; m >>= 1) x = x + __shfl_xor(x, m);
  return x;
}
template <int LPE>
__device__ __forceinline__ uint64_t ev_lanes_bits(uint64_t ballot, int sub) {
  if constexpr (LPE == 64) return ballot;
  else return (ballot >> (sub * LPE)) & ((1ull << LPE) - 1ull);
}
constexpr int ev_lanes_passes(int W) { return W >= 8 ? 1 : 8 / W; }
template <int LPE, int W, int MODE, class S, class Mt>
__global__ void __launch_bounds__(kBlock) k_ev_lanes(pgw_ev_params p, pgw_ev_step_info s, int64_t n, Mt act,
                                                     const double* __restrict__ endp, S* __restrict__ req,
                                                     uint64_t* __restrict__ chg, Mt obs, S* __restrict__ rp,
                                                     S* __restrict__ rew) {
  static_assert(LPE == 64 || W == 1, "fewer lanes than a wave per env: one word");
  constexpr int EPW = 64 / LPE, VP = LPE * W, NP = ev_lanes_passes(W);
  const int lane = threadIdx.x & 63, sub = lane / LPE, j = lane % LPE;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t e0 = wave * (NP * EPW);
  // the vehicles' shared data (the same in every pass): time left and its
  // reciprocal, scanned and parked bits
  double tl[W], rc[W];
  bool inw[W], win[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const int v = w * 64 + j, b = v & 63;
    inw[w] = v < p.n_vehicles && ((s.scan[w] >> b) & 1ull);
    win[w] = (s.window[w] >> b) & 1ull;
    tl[w] = rc[w] = 0.0;
    if constexpr (MODE == kEvTable) {
      if (inw[w]) {
        const double2 q = reinterpret_cast<const double2*>(s.tl_rcp)[v];
        tl[w] = q.x;
        rc[w] = q.y;
      }
    } else if constexpr (MODE == kEvDivide) {
      if (inw[w]) tl[w] = (endp[v] - s.time) / 60.0;
    }
  }
  // every pass's loads before any use
  double r[NP][W], a[NP], tlp[NP][W];               // (tlp: kEvPerEnv's time left, per env)
  uint64_t prev[NP][W];
  bool pw[NP][W];                                    // (kEvPerEnv: parked, per env)
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int64_t e = e0 + i * EPW + sub;
    const bool ok = e < n;
    a[i] = ok ? ev_act(s, e, act) : 0.0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const int v = w * 64 + j;
      const bool in = ok && inw[w];
      r[i][w] = in ? (double)req[e * VP + v] : 0.0;
      prev[i][w] = ok ? chg[(int64_t)w * n + e] : 0ull;
      pw[i][w] = win[w];
      tlp[i][w] = tl[w];
      if constexpr (MODE == kEvPerEnv) {
        if (in) {
          const double en = s.env_endp[e * VP + v];
          pw[i][w] = (s.time >= s.env_start[e * VP + v]) && (s.time <= floor(en));
          tlp[i][w] = (en - s.time) / 60.0;
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int64_t e = e0 + i * EPW + sub;
    const bool ok = e < n;
    const double kwh = ev_kwh_of(p, a[i]);
    double demand = 0.0, consumed = 0.0, dsum = 0.0, unserved = 0.0;
    int nact = 0, dcnt = 0;
    uint64_t now[W];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const int v = w * 64 + j, b = v & 63;
      const bool in = ok && inw[w];
      const double rr = r[i][w];
      const double tlv = tlp[i][w];
      const bool act_v = in && pw[i][w] && (rr > 0.0);
      const bool chg_v = act_v && (tlv > 0.0);
      const bool dep_v = in && !act_v && ((prev[i][w] >> b) & 1ull);
      double df;
      if constexpr (MODE == kEvTable) df = pymax(0.0, p.rate - exact_div(rr, tlv, rc[w]));
      else df = pymax(0.0, p.rate - rr / tlv);
      const double cv = pymin(kwh, rr);
      if (chg_v) req[e * VP + v] = (S)(rr - cv);
      demand = act_v ? demand + rr : demand;
      consumed = chg_v ? consumed + cv : consumed;
      dsum = chg_v ? dsum + df : dsum;
      unserved = dep_v ? unserved + rr : unserved;
      const uint64_t ba = ev_lanes_bits<LPE>(__ballot(act_v), sub);
      const uint64_t bc = ev_lanes_bits<LPE>(__ballot(chg_v), sub);
      now[w] = ba;
      nact += __builtin_popcountll(ba);
      dcnt += __builtin_popcountll(bc);
    }
    EvSums t;
    t.demand = ev_lanes_sum<LPE>(demand);
    t.consumed = ev_lanes_sum<LPE>(consumed);
    t.dsum = ev_lanes_sum<LPE>(dsum);
    t.unserved = ev_lanes_sum<LPE>(unserved);
    t.nact = nact;
    t.dcnt = dcnt;
    if (ok && j == 0) {
#pragma unroll
      for (int w = 0; w < W; ++w) chg[(int64_t)w * n + e] = now[w];
      ev_note(p, a[i]);
      (void)ev_finish(p, s, e, t, obs, rp, rew);
    }
  }
}

// ====================================================================== fused MC step
// One component of an MC agent for env e; writes its real power (and its
// reward where it has one) to the component's own buffers.
// `V`: the step's shared values -- the launch's own fields (pgw_mc_step_args)
// or a device-clocked record (pgw_mc_step_dyn); both name them alike.
// Args: pgw_mc_step_args (fp64 storage) or pgw_mc_step_args_f32 (fp32 storage).
template <class Args> struct McStore {
  using S = double;
  using Mt = pgw_mat;
};
template <> struct McStore<pgw_mc_step_args_f32> {
  using S = float;
  using Mt = pgw_matf;
};
static_assert(sizeof(pgw_mc_step_args_f32) == sizeof(pgw_mc_step_args), "pgw_mc_step_args_f32 layout");

template <bool STD, bool TR, class Args, class V, class Comp>
__device__ __forceinline__ RpRew mc_component(const Args& a, const V& v, const Comp& C,
                                              const BldDerived& d, int64_t n, int64_t e) {
  using S = typename McStore<Args>::S;
  using Mt = typename McStore<Args>::Mt;
  switch (C.kind) {
    case PGW_MC_BUILDING: {
      double fresh = 0.0;
      const S pc = (S)building_step_env<STD, S, Mt, TR>(a.bld, d, v.bld_ex_t, v.bld_ex_next, n, e, C.action,
                                                    a.bld_x, C.real_power, (S*)nullptr, a.bld_reward_state,
                                                    0, a.bld_ext, C.obs, &fresh);
      return {(double)pc, fresh};
    }
    case PGW_MC_PV: {
      const S r = (S)pv_step_env(a.pv, e, v.pv_pmax, C.action, a.pv_min_voltage, C.obs);
      C.real_power[e] = r;
      return {(double)r, 0.0};
    }
    case PGW_MC_STORAGE: {
      const S r = (S)battery_step_env(a.bat, e, C.action, a.bat_soc, C.obs);
      C.real_power[e] = r;
      return {(double)r, 0.0};
    }
    default:
      return ev_step_env(a.ev, v.ev_step, n, e, C.action, a.ev_endp, a.ev_req, a.ev_charging, C.obs,
                         C.real_power, a.ev_reward);
  }
}

// MultiComponentEnv.step (base.py:114-139) of an agent made of building / PV /
// storage / EV components (each at most once, any order): every component's
// step in order, then real power and reward summed in order from 0 -- the
// generic path's kernels and k_agent_reduce in one launch.  (Measured and
// dropped: the components as parallel blocks with the last one per env block
// forming the sums -- the device-scope release/acquire fences that make the
// other blocks' outputs visible across XCDs write back L2 and cost more than
// the overlap gains: C3 19.7 -> 34.6 us.)
//
// Layout: a block of n_comp waves serves 64 envs, wave w running component slot
// w for all of them.  The components of an agent are independent within a step
// (each reads only its own action and state), so they run side by side on the
// block's SIMDs instead of one after another in each lane; each wave leaves its
// component's real power and reward in LDS and, after the block barrier, wave 0
// forms the sums in component order -- the same values and the same operation
// order as one lane doing everything, without any cross-block synchronisation.
//
// CLK (pgw_mc_step_args.clock != NULL): the step's shared values come from the
// device table dyn[k], k = this block's clock -- the launch's arguments are
// then the same at every step (hipGraph replay).  One clock per block: each is
// read and advanced by its own block only (plain loads and stores, ordered by
// the kernel boundary), so there is no cross-block count to contend on (one
// counter advanced by the last block to retire cost 2.3 us per step: 256
// serialised device-scope atomics).
//
// Split EV (blockDim.x > 64 n_comp: the launch added kEvGroups - 1 waves): the
// EV slot's vehicle walk is shared by kEvGroups waves of the block, each over
// one group of chunks (ev_walk), with the charging bits ORed in LDS; the last
// group wave to finish its walk (an LDS arrival count, acquire-release at
// workgroup scope) folds the partial sums in group order and finishes the EV
// step -- without waiting for the building wave, as a block barrier would.
// C3 runs one block per CU; the phase trace (tools/gpu/mc_trace.py) showed the
// walk groups (about 2 us per chunk each) as the critical path at midday and
// the building wave plus the fold behind a barrier at night.
template <class Args, bool STD, bool CLK, bool TR = false>
__global__ void __launch_bounds__(64 * (4 + kEvGroups - 1)) k_mc_step(Args a_, BldDerived d, int64_t n) {
  using S = typename McStore<Args>::S;
  const Args& a = PGW_KERNARG0(Args);
  long long* const tr = TR ? g_mc_trace : nullptr;
  mc_trace<TR>(tr, 0);
  __shared__ double s_rp[4][64], s_rew[4][64];
  __shared__ uint64_t s_bits[PGW_EV_MAX_WORDS * 64];
  __shared__ double s_evs[kEvGroups][4][64];
  __shared__ int s_evc[kEvGroups][2][64];
  __shared__ int s_arrive, s_done;
  __shared__ pgw_building_params s_bp;                // the building wave's parameters (bld_stage_wave)
  __shared__ BldDerived s_bd;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // component slot
  const int lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * 64 + lane;
  const bool split = (int)(blockDim.x >> 6) > a.n_comp;                   // (uniform)
  int ev_slot = 0;
  for (int c = 0; c < a.n_comp; ++c) ev_slot = a.comp[c].kind == PGW_MC_EV ? c : ev_slot;
  if (split) {
    for (int i = threadIdx.x; i < PGW_EV_MAX_WORDS * 64; i += blockDim.x) s_bits[i] = 0ull;
    if (threadIdx.x == 0) s_arrive = s_done = 0;
  }
  // CLK: the step's record staged in LDS by the block (80 doubles): its
  // fields are then read at fixed LDS addresses, with no pointer to keep live
  // (a pointer into the table costs SGPRs the step does not have)
  __shared__ pgw_mc_step_dyn s_dyn;
  int k = 0;
  if constexpr (CLK) {
    constexpr int kWords = (int)(sizeof(pgw_mc_step_dyn) / sizeof(double));
    k = a.clock[blockIdx.x];
    const int r = min(max(k, 0), a.n_dyn - 1);
    for (int i = threadIdx.x; i < kWords; i += blockDim.x)      // (a block is 1-7 waves)
      reinterpret_cast<double*>(&s_dyn)[i] = reinterpret_cast<const double*>(a.dyn + r)[i];
  }
  if (CLK || split) __syncthreads();
  mc_trace<TR>(tr, 1);
  const pgw_ev_step_info& evs = CLK ? s_dyn.ev_step : a.ev_step;
  const bool ev_wave = split && (w >= a.n_comp || w == ev_slot);
  if (ev_wave) {
    const int g = w >= a.n_comp ? w - a.n_comp + 1 : 0;
    if (e < n) {
      const EvSums t = ev_step_group<S, typename McStore<Args>::Mt, TR>(a.ev, evs, n, e, a.comp[ev_slot].action,
                                                                        a.ev_endp, a.ev_req, a.ev_charging, g,
                                                                        s_bits, lane);
      s_evs[g][0][lane] = t.demand;
      s_evs[g][1][lane] = t.consumed;
      s_evs[g][2][lane] = t.dsum;
      s_evs[g][3][lane] = t.unserved;
      s_evc[g][0][lane] = t.dcnt;
      s_evc[g][1][lane] = t.nact;
    }
    mc_trace<TR>(tr, 2);
    // arrival: this wave's partials and charging bits (LDS) are released to
    // the wave that arrives last, which acquires them and finishes the step
    int prior = 0;
    if (lane == 0)
      prior = __hip_atomic_fetch_add(&s_arrive, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    prior = __builtin_amdgcn_readfirstlane(prior);
    if (prior == kEvGroups - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      if (e < n) {
        EvSums t{0.0, 0.0, 0.0, 0.0, 0, 0};
#pragma unroll
        for (int q = 0; q < kEvGroups; ++q) {
          t.demand = t.demand + s_evs[q][0][lane];
          t.consumed = t.consumed + s_evs[q][1][lane];
          t.dsum = t.dsum + s_evs[q][2][lane];
          t.unserved = t.unserved + s_evs[q][3][lane];
          t.dcnt += s_evc[q][0][lane];
          t.nact += s_evc[q][1][lane];
        }
        for (int j = 0; j < evs.n_words; ++j) a.ev_charging[(int64_t)j * n + e] = s_bits[j * 64 + lane];
        const auto& C = a.comp[ev_slot];
        const RpRew r = ev_finish(a.ev, evs, e, t, C.obs, C.real_power, a.ev_reward);
        s_rp[ev_slot][lane] = r.rp;
        s_rew[ev_slot][lane] = r.rew;
      }
      mc_trace<TR>(tr, 4);
    }
  } else if (STD && a.comp[w].kind == PGW_MC_BUILDING) {   // (uniform) the std building: bld_wave_std
    using Mt = typename McStore<Args>::Mt;
    const auto& C = a.comp[w];
    const pgw_building_exo& ex = CLK ? s_dyn.bld_ex_t : a.bld_ex_t;
    const pgw_building_exo& exn = CLK ? s_dyn.bld_ex_next : a.bld_ex_next;
    const RpRew r = bld_wave_std<S, Mt, TR>(a.bld, d, s_bp, s_bd, ex, exn, n, e, C.action, a.bld_x,
                                            C.real_power, a.bld_reward_state, C.obs);
    if (e < n) {
      s_rp[w][lane] = r.rp;
      s_rew[w][lane] = r.rew;
    }
    mc_trace<TR>(tr, 2);
  } else {
    if (e < n) {
      const auto& C = a.comp[w];
      RpRew r;
      if constexpr (CLK)
        r = mc_component<STD, TR>(a, s_dyn, C, d, n, e);
      else
        r = mc_component<STD, TR>(a, a, C, d, n, e);
      s_rp[w][lane] = r.rp;
      s_rew[w][lane] = r.rew;
    }
    mc_trace<TR>(tr, 2);
  }
  // the sums: split blocks let the wave that finishes last form them (an
  // arrival count as for the EV fold), so the light waves leave at once
  // instead of waiting at a barrier for the walk; unsplit ones use wave 0
  if (split) {
    int prior = 0;
    if (lane == 0) prior = __hip_atomic_fetch_add(&s_done, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    prior = __builtin_amdgcn_readfirstlane(prior);
    if (prior != (int)(blockDim.x >> 6) - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  } else {
    __syncthreads();
  }
  mc_trace<TR>(tr, 5);
  // (every wave read k before the staging barrier)
  if (CLK && lane == 0 && (split || w == 0)) a.clock[blockIdx.x] = k + 1;
  if ((!split && w != 0) || e >= n) return;
  double rp_sum = 0.0, rew_sum = 0.0;
  for (int c = 0; c < a.n_comp; ++c) {
    rp_sum = rp_sum + s_rp[c][lane];
    rew_sum = rew_sum + s_rew[c][lane];
  }
  a.real_power[e] = (S)rp_sum;
  a.reward[e] = (S)rew_sum;
  mc_trace<TR>(tr, 6);
}

// ====================================================================== fused multi-agent step
// MultiAgentEnv.step (multiagent_env.py:151-212) of MC-kind agents, e.g. the
// heterogeneous scenario (scenarios/heterogeneous.py:13-112): a block of
// n_comp waves serves 64 envs, wave w running component slot w (k_mc_step's
// layout, widened to every agent's components: the components of all agents
// are independent within a step -- each reads only its own action and state
// and the PREVIOUS power flow's voltages).  After the block barrier wave 0
// forms each MultiComponentEnv agent's sums in component order (base.py:125-156)
// and each bus's load in agent order (multiagent_env.py:171-181), the values and
// operation order of pgw_agent_reduce.
//
// Waves: the building and the EV (the long per-env chains) get a wave each and
// the light PV / storage slots share one (pgw_ma_step_args.wave_*): a wave per
// slot made the heterogeneous scenario's blocks 5 waves, which at the kernel's
// register count did not all fit at once.
// The agents' and buses' part of pgw_ma_step_args (n_agents .. bus_p), as laid
// out there: copied whole into LDS for the sums.
struct MaSums {
  int32_t n_agents, n_bus;
  int32_t first[PGW_MAX_AGENTS], count[PGW_MAX_AGENTS];
  int32_t bus[PGW_MAX_AGENTS], sum[PGW_MAX_AGENTS];
  double* rp[PGW_MAX_AGENTS];
  double* rew[PGW_MAX_AGENTS];
  double* bus_p;
};
static_assert(offsetof(pgw_ma_step_args, n_waves) - offsetof(pgw_ma_step_args, n_agents) == sizeof(MaSums) &&
              offsetof(pgw_ma_step_args, n_agents) % 8 == 0 && sizeof(MaSums) % 8 == 0 && sizeof(MaSums) / 8 <= 64,
              "MaSums mirrors pgw_ma_step_args");
static_assert(offsetof(pgw_ma_step_args, agent_first) - offsetof(pgw_ma_step_args, n_agents) == offsetof(MaSums, first) &&
              offsetof(pgw_ma_step_args, agent_sum) - offsetof(pgw_ma_step_args, n_agents) == offsetof(MaSums, sum) &&
              offsetof(pgw_ma_step_args, agent_real_power) - offsetof(pgw_ma_step_args, n_agents) == offsetof(MaSums, rp) &&
              offsetof(pgw_ma_step_args, bus_p) - offsetof(pgw_ma_step_args, n_agents) == offsetof(MaSums, bus_p),
              "MaSums field offsets");

// (3 waves per SIMD at least: the heterogeneous scenario's 1 024 three-wave
// blocks then all fit at once, 4 per CU; at 2 they ran in two rounds)
template <bool STD, bool TR = false>
__global__ void __launch_bounds__(64 * PGW_MA_MAX_SLOTS) __attribute__((amdgpu_waves_per_eu(3))) k_ma_step(pgw_ma_step_args a_, BldDerived d,
                                                                   int64_t n) {
  const pgw_ma_step_args& a = PGW_KERNARG0(pgw_ma_step_args);
  long long* const tr = TR ? g_mc_trace : nullptr;
  mc_trace<TR>(tr, 0);
  __shared__ double s_rp[PGW_MA_MAX_SLOTS][64], s_rew[PGW_MA_MAX_SLOTS][64];
  __shared__ pgw_building_params s_bp;                // the building wave's parameters (bld_stage_wave)
  __shared__ BldDerived s_bd;
  __shared__ MaSums s_sums;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  // the sums' plan (agents' slots, buses, output pointers), read by wave 0
  // after the barrier: staged here by the block's last wave (not the
  // building's), so the tail is LDS reads, not ~40 waited scalar loads
  if (wv == (int)(blockDim.x >> 6) - 1) {
    constexpr int kW = (int)(sizeof(MaSums) / 8);
    const int l = (int)(threadIdx.x & 63);
    if (l < kW) reinterpret_cast<uint64_t*>(&s_sums)[l] = reinterpret_cast<const uint64_t*>(&a.n_agents)[l];
  }
  const int lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * 64 + lane;
  // the wave's role, uniform: a building or an EV slot runs alone in its wave,
  // the light PV / storage slots one after another (a loop over every kind let
  // the compiler hoist all parameter loads of every path into one prologue,
  // spilling SGPRs: 10 us for a PV-only step)
  const int c0 = a.wave_slot[a.wave_first[wv]];
  const int kind0 = a.comp[c0].kind;
  if (STD && kind0 == PGW_MC_BUILDING) {           // (uniform) every lane stages: bld_wave_std
    const pgw_mc_component& C = a.comp[c0];
    const RpRew r = bld_wave_std<double, pgw_mat, TR>(a.bld, d, s_bp, s_bd, a.bld_ex_t, a.bld_ex_next, n, e,
                                                      C.action, a.bld_x, C.real_power, a.bld_reward_state, C.obs);
    if (e < n) {
      s_rp[c0][lane] = r.rp;
      s_rew[c0][lane] = r.rew;                      // the fresh reward (MC semantics)
    }
  } else if (e < n) {
    if (kind0 == PGW_MC_BUILDING) {
      const pgw_mc_component& C = a.comp[c0];
      double fresh = 0.0;                             // the fresh reward (MC semantics)
      s_rp[c0][lane] = building_step_env<STD, double, pgw_mat, TR>(a.bld, d, a.bld_ex_t, a.bld_ex_next, n, e,
                                                                   C.action, a.bld_x, C.real_power, nullptr,
                                                                   a.bld_reward_state, 0, a.bld_ext, C.obs,
                                                                   &fresh);
      s_rew[c0][lane] = fresh;
    } else if (kind0 == PGW_MC_EV) {
      const pgw_mc_component& C = a.comp[c0];
      const RpRew r = ev_step_env(a.ev, a.ev_step, n, e, C.action, a.ev_endp, a.ev_req, a.ev_charging, C.obs,
                                  C.real_power, a.ev_reward);
      s_rp[c0][lane] = r.rp;
      s_rew[c0][lane] = r.rew;
    } else {
      // the light slots in two passes: every slot's loads (action, SoC or the
      // min voltage) go out before any slot's stores -- one slot after another
      // each waited for the previous slot's stores too (vmcnt is in order):
      // three round trips where one does (HET's PV farm, building PV, storage)
      const int cnt = a.wave_count[wv], first = a.wave_first[wv];
      double act_v[PGW_MA_MAX_SLOTS], st_v[PGW_MA_MAX_SLOTS];
#pragma unroll
      for (int i = 0; i < PGW_MA_MAX_SLOTS; ++i) {
        if (i >= cnt) break;
        const int w = a.wave_slot[first + i];
        const pgw_mc_component& C = a.comp[w];
        act_v[i] = C.action.ptr ? ld(C.action, e, 0) : 0.0;
        if (C.kind == PGW_MC_PV) {
          const bool two = a.slot_pv2[w] != 0;
          const double* vmin = two ? a.pv2_min_voltage : a.pv_min_voltage;
          st_v[i] = ((two ? a.pv2 : a.pv).grid_aware || a.slot_reward[w]) ? vmin[e] : 0.0;
        } else {
          st_v[i] = a.bat_soc[e];
        }
      }
#pragma unroll
      for (int i = 0; i < PGW_MA_MAX_SLOTS; ++i) {
        if (i >= cnt) break;
        const int w = a.wave_slot[first + i];
        const pgw_mc_component& C = a.comp[w];
        double rp, rew = 0.0;
        if (C.kind == PGW_MC_PV) {                    // pv_step_env on the loaded values
          const bool two = a.slot_pv2[w] != 0;
          const pgw_pv_params& pp = two ? a.pv2 : a.pv;
          const double pmax = two ? a.pv2_pmax : a.pv_pmax;
          const double x = st_v[i];
          st(C.obs, e, 0, pv_obs(pp, pmax));
          if (pp.grid_aware) st(C.obs, e, 1, pp.rescale ? to_scaled(x, pp.vmin_low, pp.vmin_high) : x);
          rp = C.action.ptr ? pv_real_power(pp, act_v[i], pmax) : 0.0;
          if (a.slot_reward[w]) {                     // ThisPVEnv.step_reward: k_band_penalty's ops
            const double l = x - a.band_lo, u = a.band_hi - x;
            const double viol = ((l < 0.0) ? l : 0.0) + ((u < 0.0) ? u : 0.0);
            const double y = a.band_scale * viol;
            rew = -(y * y);
            a.slot_reward[w][e] = rew;
          }
        } else {                                      // battery_step_env on the loaded values
          double soc = st_v[i];
          const double power = battery_step(a.bat, act_v[i], soc);
          a.bat_soc[e] = soc;
          st(C.obs, e, 0, battery_obs(a.bat, soc));
          rp = -power;
        }
        C.real_power[e] = rp;
        s_rp[w][lane] = rp;
        s_rew[w][lane] = rew;
      }
    }
  }
  mc_trace<TR>(tr, 2);
  __syncthreads();
  mc_trace<TR>(tr, 5);
  if (wv != 0 || e >= n) return;
  const MaSums& m = s_sums;
  double ap[PGW_MAX_AGENTS];
#pragma unroll
  for (int g = 0; g < PGW_MAX_AGENTS; ++g) {     // (constant indices: ap stays in registers)
    ap[g] = 0.0;
    if (g >= m.n_agents) continue;
    const int c0 = m.first[g];
    if (m.sum[g]) {
      double rp_sum = 0.0, rew_sum = 0.0;
      for (int c = c0; c < c0 + m.count[g]; ++c) {
        rp_sum = rp_sum + s_rp[c][lane];
        rew_sum = rew_sum + s_rew[c][lane];
      }
      m.rp[g][e] = rp_sum;
      m.rew[g][e] = rew_sum;
      ap[g] = rp_sum;
    } else {
      ap[g] = s_rp[c0][lane];
    }
  }
  for (int b = 0; b < m.n_bus; ++b) {
    double acc = 0.0;
#pragma unroll
    for (int g = 0; g < PGW_MAX_AGENTS; ++g)
      acc = (g < m.n_agents && m.bus[g] == b) ? acc + ap[g] : acc;
    m.bus_p[(int64_t)b * n + e] = acc;
  }
  mc_trace<TR>(tr, 6);
}

// ====================================================================== MC reduce
__global__ void __launch_bounds__(kBlock) k_agent_reduce(pgw_reduce_args a, int64_t n,
                                                         double* __restrict__ rp,
                                                         double* __restrict__ rew) {
  int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  double r = 0.0, w = 0.0;
  for (int c = 0; c < a.n_comp; ++c) {
    r = r + (a.reward[c] ? a.reward[c][e] : 0.0);
    w = w + (a.real_power[c] ? a.real_power[c][e] : 0.0);
  }
  if (rp) rp[e] = w;
  if (rew) rew[e] = r;
}

}  // namespace pgw

using namespace pgw;

// pgw_mc_ev_split_mode: -1 auto, 0 one lane, 1 split.  Initialised once at load
// from PGW_MC_EV_SPLIT (A/B scripts); the step reads the atomic, never the
// environment.
static int initial_ev_split_mode() {
  const char* v = getenv("PGW_MC_EV_SPLIT");
  return (v && (v[0] == '0' || v[0] == '1')) ? v[0] - '0' : -1;
}
static std::atomic<int> g_mc_ev_split{initial_ev_split_mode()};
// pgw_debug_mc_trace: set -> the MC / multi-agent steps launch their TR kernels
static std::atomic<bool> g_mc_trace_on{false};

#define PGW_LAUNCH(kernel, n, stream, ...)                                         \
  do {                                                                                 \
    if ((n) > 0)                                                                       \
      hipLaunchKernelGGL(kernel, dim3(grid_for(n)), dim3(kBlock), 0,                   \
                         (hipStream_t)(stream), __VA_ARGS__);                          \
    return check_launch(#kernel);                                                      \
  } while (0)

extern "C" {

int32_t pgw_abi_version(void) { return PGW_ABI_VERSION; }
const char* pgw_last_error(void) { return g_err; }

int32_t pgw_battery_reset(const pgw_battery_params* p, int64_t n, const double* init, double* soc,
                          pgw_mat obs, void* stream) {
  PGW_REQUIRE(p && init && soc && obs.ptr && n >= 0, "pgw_battery_reset: null argument");
  PGW_LAUNCH((k_battery_reset<double, pgw_mat>), n, stream, *p, n, init, soc, obs);
}

int32_t pgw_battery_reset_f32(const pgw_battery_params* p, int64_t n, const float* init, float* soc,
                              pgw_matf obs, void* stream) {
  PGW_REQUIRE(p && init && soc && obs.ptr && n >= 0, "pgw_battery_reset_f32: null argument");
  PGW_LAUNCH((k_battery_reset<float, pgw_matf>), n, stream, *p, n, init, soc, obs);
}

int32_t pgw_battery_step(const pgw_battery_params* p, int64_t n, pgw_mat action, double* soc,
                         pgw_mat obs, double* real_power, void* stream) {
  PGW_REQUIRE(p && action.ptr && soc && obs.ptr && real_power && n >= 0,
              "pgw_battery_step: null argument");
  PGW_LAUNCH((k_battery_step<double, pgw_mat>), n, stream, *p, n, action, soc, obs, real_power);
}

int32_t pgw_battery_step_f32(const pgw_battery_params* p, int64_t n, pgw_matf action, float* soc,
                             pgw_matf obs, float* real_power, void* stream) {
  PGW_REQUIRE(p && action.ptr && soc && obs.ptr && real_power && n >= 0,
              "pgw_battery_step_f32: null argument");
  PGW_LAUNCH((k_battery_step<float, pgw_matf>), n, stream, *p, n, action, soc, obs, real_power);
}

int32_t pgw_pv_obs(const pgw_pv_params* p, int64_t n, double pmax, const double* min_voltage,
                   pgw_mat obs, void* stream) {
  PGW_REQUIRE(p && obs.ptr && n >= 0, "pgw_pv_obs: null argument");
  PGW_REQUIRE(!p->grid_aware || min_voltage, "pgw_pv_obs: grid_aware needs min_voltage");
  pgw_mat none{nullptr, 0, 0};
  PGW_LAUNCH((k_pv<double, pgw_mat>), n, stream, *p, n, pmax, none, min_voltage, obs, (double*)nullptr);
}

int32_t pgw_pv_obs_f32(const pgw_pv_params* p, int64_t n, double pmax, const double* min_voltage,
                       pgw_matf obs, void* stream) {
  PGW_REQUIRE(p && obs.ptr && n >= 0, "pgw_pv_obs_f32: null argument");
  PGW_REQUIRE(!p->grid_aware || min_voltage, "pgw_pv_obs_f32: grid_aware needs min_voltage");
  pgw_matf none{nullptr, 0, 0};
  PGW_LAUNCH((k_pv<float, pgw_matf>), n, stream, *p, n, pmax, none, min_voltage, obs, (float*)nullptr);
}

int32_t pgw_pv_step_f32(const pgw_pv_params* p, int64_t n, double pmax, pgw_matf action,
                        const double* min_voltage, pgw_matf obs, float* real_power, void* stream) {
  PGW_REQUIRE(p && action.ptr && obs.ptr && real_power && n >= 0, "pgw_pv_step_f32: null argument");
  PGW_REQUIRE(!p->grid_aware || min_voltage, "pgw_pv_step_f32: grid_aware needs min_voltage");
  PGW_LAUNCH((k_pv<float, pgw_matf>), n, stream, *p, n, pmax, action, min_voltage, obs, real_power);
}

int32_t pgw_pv_step(const pgw_pv_params* p, int64_t n, double pmax, pgw_mat action,
                    const double* min_voltage, pgw_mat obs, double* real_power, void* stream) {
  PGW_REQUIRE(p && action.ptr && obs.ptr && real_power && n >= 0, "pgw_pv_step: null argument");
  PGW_REQUIRE(!p->grid_aware || min_voltage, "pgw_pv_step: grid_aware needs min_voltage");
  PGW_LAUNCH((k_pv<double, pgw_mat>), n, stream, *p, n, pmax, action, min_voltage, obs, real_power);
}

int32_t pgw_building_reset(const pgw_building_params* p, const pgw_building_exo* ex0, int64_t n,
                           double* x, double* p_consumed, double* reward_state,
                           pgw_building_ext ext, pgw_mat obs, void* stream) {
  PGW_REQUIRE(p && ex0 && x && p_consumed && obs.ptr && n >= 0, "pgw_building_reset: null argument");
  PGW_REQUIRE(p->n_obs >= 0 && p->n_obs <= PGW_BLD_MAX_OBS, "pgw_building_reset: bad n_obs");
  PGW_LAUNCH((k_building_reset<double, pgw_mat>), n, stream, *p, *ex0, n, x, p_consumed, reward_state, ext, obs);
}

int32_t pgw_building_reset_f32(const pgw_building_params* p, const pgw_building_exo* ex0, int64_t n,
                               float* x, float* p_consumed, float* reward_state,
                               pgw_building_ext ext, pgw_matf obs, void* stream) {
  PGW_REQUIRE(p && ex0 && x && p_consumed && obs.ptr && n >= 0, "pgw_building_reset_f32: null argument");
  PGW_REQUIRE(p->n_obs >= 0 && p->n_obs <= PGW_BLD_MAX_OBS, "pgw_building_reset_f32: bad n_obs");
  PGW_LAUNCH((k_building_reset<float, pgw_matf>), n, stream, *p, *ex0, n, x, p_consumed, reward_state, ext, obs);
}

int32_t pgw_building_step(const pgw_building_params* p, const pgw_building_exo* ex_t,
                          const pgw_building_exo* ex_next, int64_t n, pgw_mat action, double* x,
                          double* p_consumed, double* reward_out, double* reward_state,
                          int32_t lagged, pgw_building_ext ext, pgw_mat obs, void* stream) {
  PGW_REQUIRE(p && ex_t && ex_next && action.ptr && x && p_consumed && obs.ptr && n >= 0,
              "pgw_building_step: null argument");
  PGW_REQUIRE(!lagged || reward_state, "pgw_building_step: lagged reward needs reward_state");
  PGW_REQUIRE(p->n_obs >= 0 && p->n_obs <= PGW_BLD_MAX_OBS, "pgw_building_step: bad n_obs");
  const BldDerived d = make_bld_derived(*p);
  if (bld_is_std(*p))
    PGW_LAUNCH((k_building_step<true, double, pgw_mat>), n, stream, *p, d, *ex_t, *ex_next, n, action, x,
               p_consumed, reward_out, reward_state, lagged, ext, obs);
  PGW_LAUNCH((k_building_step<false, double, pgw_mat>), n, stream, *p, d, *ex_t, *ex_next, n, action, x,
             p_consumed, reward_out, reward_state, lagged, ext, obs);
}

int32_t pgw_building_step_f32(const pgw_building_params* p, const pgw_building_exo* ex_t,
                              const pgw_building_exo* ex_next, int64_t n, pgw_matf action, float* x,
                              float* p_consumed, float* reward_out, float* reward_state,
                              int32_t lagged, pgw_building_ext ext, pgw_matf obs, void* stream) {
  PGW_REQUIRE(p && ex_t && ex_next && action.ptr && x && p_consumed && obs.ptr && n >= 0,
              "pgw_building_step_f32: null argument");
  PGW_REQUIRE(!lagged || reward_state, "pgw_building_step_f32: lagged reward needs reward_state");
  PGW_REQUIRE(p->n_obs >= 0 && p->n_obs <= PGW_BLD_MAX_OBS, "pgw_building_step_f32: bad n_obs");
  const BldDerived d = make_bld_derived(*p);
  if (bld_is_std(*p))
    PGW_LAUNCH((k_building_step<true, float, pgw_matf>), n, stream, *p, d, *ex_t, *ex_next, n, action, x,
               p_consumed, reward_out, reward_state, lagged, ext, obs);
  PGW_LAUNCH((k_building_step<false, float, pgw_matf>), n, stream, *p, d, *ex_t, *ex_next, n, action, x,
             p_consumed, reward_out, reward_state, lagged, ext, obs);
}

int32_t pgw_ev_reset(const pgw_ev_params* p, int64_t n, const double* req0, double* req,
                     uint64_t* charging, void* stream) {
  PGW_REQUIRE(p && req0 && req && charging && n >= 0, "pgw_ev_reset: null argument");
  PGW_REQUIRE(p->n_vehicles >= 0 && p->n_vehicles <= 64 * PGW_EV_MAX_WORDS,
              "pgw_ev_reset: too many vehicles");
  int32_t W = (p->n_vehicles + 63) / 64;
  PGW_LAUNCH(k_ev_reset<double>, n, stream, n, p->n_vehicles, W, req0, req, charging);
}

int32_t pgw_ev_reset_f32(const pgw_ev_params* p, int64_t n, const double* req0, float* req,
                         uint64_t* charging, void* stream) {
  PGW_REQUIRE(p && req0 && req && charging && n >= 0, "pgw_ev_reset_f32: null argument");
  PGW_REQUIRE(p->n_vehicles >= 0 && p->n_vehicles <= 64 * PGW_EV_MAX_WORDS,
              "pgw_ev_reset_f32: too many vehicles");
  int32_t W = (p->n_vehicles + 63) / 64;
  PGW_LAUNCH(k_ev_reset<float>, n, stream, n, p->n_vehicles, W, req0, req, charging);
}

int32_t pgw_ev_reset_tables(const pgw_ev_params* p, int64_t n, const double* req0_env, double* req,
                            uint64_t* charging, void* stream) {
  PGW_REQUIRE(p && req0_env && req && charging && n >= 0, "pgw_ev_reset_tables: null argument");
  PGW_REQUIRE(p->n_vehicles >= 0 && p->n_vehicles <= 64 * PGW_EV_MAX_WORDS,
              "pgw_ev_reset_tables: too many vehicles");
  const int32_t W = (p->n_vehicles + 63) / 64;
  PGW_LAUNCH(k_ev_reset_tables<double>, n, stream, n, p->n_vehicles, W, req0_env, req, charging);
}

int32_t pgw_ev_reset_tables_f32(const pgw_ev_params* p, int64_t n, const double* req0_env, float* req,
                                uint64_t* charging, void* stream) {
  PGW_REQUIRE(p && req0_env && req && charging && n >= 0, "pgw_ev_reset_tables_f32: null argument");
  PGW_REQUIRE(p->n_vehicles >= 0 && p->n_vehicles <= 64 * PGW_EV_MAX_WORDS,
              "pgw_ev_reset_tables_f32: too many vehicles");
  const int32_t W = (p->n_vehicles + 63) / 64;
  PGW_LAUNCH(k_ev_reset_tables<float>, n, stream, n, p->n_vehicles, W, req0_env, req, charging);
}

int32_t pgw_ev_step(const pgw_ev_params* p, const pgw_ev_step_info* s, int64_t n, pgw_mat action,
                    const double* endp, double* req, uint64_t* charging, pgw_mat obs,
                    double* real_power, double* reward, void* stream) {
  PGW_REQUIRE(p && s && endp && req && charging && obs.ptr && real_power && reward && n >= 0,
              "pgw_ev_step: null argument");
  PGW_REQUIRE(s->n_words == (p->n_vehicles + 63) / 64 && s->n_words <= PGW_EV_MAX_WORDS,
              "pgw_ev_step: n_words does not match n_vehicles");
  PGW_REQUIRE(!s->env_start == !s->env_endp && (!s->env_start || !s->tl_rcp),
              "pgw_ev_step: per-env tables need env_start and env_endp, and no tl_rcp");
  PGW_LAUNCH((k_ev_step<double, pgw_mat>), n, stream, *p, *s, n, action, endp, req, charging, obs, real_power,
             reward);
}

int32_t pgw_ev_step_f32(const pgw_ev_params* p, const pgw_ev_step_info* s, int64_t n, pgw_matf action,
                        const double* endp, float* req, uint64_t* charging, pgw_matf obs,
                        float* real_power, float* reward, void* stream) {
  PGW_REQUIRE(p && s && endp && req && charging && obs.ptr && real_power && reward && n >= 0,
              "pgw_ev_step_f32: null argument");
  PGW_REQUIRE(s->n_words == (p->n_vehicles + 63) / 64 && s->n_words <= PGW_EV_MAX_WORDS,
              "pgw_ev_step_f32: n_words does not match n_vehicles");
  PGW_REQUIRE(!s->env_start == !s->env_endp && (!s->env_start || !s->tl_rcp),
              "pgw_ev_step_f32: per-env tables need env_start and env_endp, and no tl_rcp");
  PGW_LAUNCH((k_ev_step<float, pgw_matf>), n, stream, *p, *s, n, action, endp, req, charging, obs, real_power,
             reward);
}

int32_t pgw_ev_row(int32_t n_vehicles) {
  if (n_vehicles <= 16) return 16;
  if (n_vehicles <= 32) return 32;
  int w = 1;
  while (64 * w < n_vehicles) w *= 2;
  return 64 * w;
}

int32_t pgw_ev_step_lanes(const pgw_ev_params* p, const pgw_ev_step_info* s, int64_t n, pgw_mat action,
                          const double* endp, double* req, uint64_t* charging, pgw_mat obs,
                          double* real_power, double* reward, void* stream) {
  PGW_REQUIRE(p && s && endp && req && charging && obs.ptr && real_power && reward && n >= 0,
              "pgw_ev_step_lanes: null argument");
  PGW_REQUIRE(s->n_words == (p->n_vehicles + 63) / 64 && s->n_words <= PGW_EV_MAX_WORDS,
              "pgw_ev_step_lanes: n_words does not match n_vehicles");
  PGW_REQUIRE(!s->env_start == !s->env_endp && (!s->env_start || !s->tl_rcp),
              "pgw_ev_step_lanes: per-env tables need env_start and env_endp, and no tl_rcp");
  if (n == 0) return PGW_OK;
  const int row = pgw_ev_row(p->n_vehicles);
  const int lpe = row < 64 ? row : 64, W = row / 64 > 0 ? row / 64 : 1;
  const int mode = s->env_start ? kEvPerEnv : s->tl_rcp ? kEvTable : kEvDivide;
  const int64_t per_wave = (int64_t)ev_lanes_passes(W) * (64 / lpe);
  const int64_t waves = (n + per_wave - 1) / per_wave;
  const dim3 grid((unsigned)((waves * 64 + kBlock - 1) / kBlock)), block(kBlock);
  hipStream_t st = (hipStream_t)stream;
#define PGW_EV_LANES(L, WW, M)                                                                             \
  hipLaunchKernelGGL((k_ev_lanes<L, WW, M, double, pgw_mat>), grid, block, 0, st, *p, *s, n, action, endp, req, \
                     charging, obs, real_power, reward)
#define PGW_EV_LANES_M(L, WW)                           \
  do {                                                  \
    if (mode == kEvTable) PGW_EV_LANES(L, WW, kEvTable);  \
    else if (mode == kEvPerEnv) PGW_EV_LANES(L, WW, kEvPerEnv); \
    else PGW_EV_LANES(L, WW, kEvDivide);                 \
  } while (0)
  if (lpe == 16) PGW_EV_LANES_M(16, 1);
  else if (lpe == 32) PGW_EV_LANES_M(32, 1);
  else if (W == 1) PGW_EV_LANES_M(64, 1);
  else if (W == 2) PGW_EV_LANES_M(64, 2);
  else if (W == 4) PGW_EV_LANES_M(64, 4);
  else if (W == 8) PGW_EV_LANES_M(64, 8);
  else PGW_EV_LANES_M(64, 16);
#undef PGW_EV_LANES_M
#undef PGW_EV_LANES
  return check_launch("k_ev_lanes");
}

int32_t pgw_debug_mc_trace(long long* buf) {
  PGW_REQUIRE(hipMemcpyToSymbol(HIP_SYMBOL(g_mc_trace), &buf, sizeof(buf)) == hipSuccess,
              "pgw_debug_mc_trace: hipMemcpyToSymbol failed");
  g_mc_trace_on.store(buf != nullptr);
  return PGW_OK;
}

int32_t pgw_mc_ev_split_mode(int32_t mode, int32_t* previous) {
  PGW_REQUIRE(mode >= -1 && mode <= 1, "pgw_mc_ev_split_mode: mode must be -1, 0 or 1");
  const int old = g_mc_ev_split.exchange(mode);
  if (previous) *previous = old;
  return PGW_OK;
}

}  // extern "C"

template <class Args>
static int32_t mc_agent_step(const Args* a, int64_t n, void* stream) {
  PGW_REQUIRE(a && n >= 0 && a->n_comp >= 1 && a->n_comp <= 4, "pgw_mc_agent_step: bad args");
  PGW_REQUIRE(a->real_power && a->reward, "pgw_mc_agent_step: null output");
  int seen = 0;
  for (int c = 0; c < a->n_comp; ++c) {
    const auto& C = a->comp[c];
    PGW_REQUIRE(C.kind >= 0 && C.kind <= 3 && !(seen & (1 << C.kind)),
                "pgw_mc_agent_step: component kinds must be distinct PGW_MC_* values");
    seen |= 1 << C.kind;
    PGW_REQUIRE(C.action.ptr && C.obs.ptr && C.real_power, "pgw_mc_agent_step: component %d buffers", c);
    if (C.kind == PGW_MC_BUILDING)
      PGW_REQUIRE(a->bld_x && a->bld_reward_state && a->bld.n_obs <= PGW_BLD_MAX_OBS,
                  "pgw_mc_agent_step: building buffers");
    if (C.kind == PGW_MC_PV) PGW_REQUIRE(!a->pv.grid_aware || a->pv_min_voltage, "pgw_mc_agent_step: min_voltage");
    if (C.kind == PGW_MC_STORAGE) PGW_REQUIRE(a->bat_soc, "pgw_mc_agent_step: storage buffers");
    if (C.kind == PGW_MC_EV)
      PGW_REQUIRE(a->ev_endp && a->ev_req && a->ev_charging && a->ev_reward &&
                  a->ev_step.n_words <= PGW_EV_MAX_WORDS &&
                  !a->ev_step.env_start == !a->ev_step.env_endp &&
                  (!a->ev_step.env_start || !a->ev_step.tl_rcp), "pgw_mc_agent_step: EV buffers");
  }
  PGW_REQUIRE(!a->clock == !a->dyn && (!a->dyn || a->n_dyn >= 1),
              "pgw_mc_agent_step: clock and dyn go together, n_dyn >= 1");
  const BldDerived d = make_bld_derived(a->bld);
  bool std_bld = false;
  for (int c = 0; c < a->n_comp; ++c)
    if (a->comp[c].kind == PGW_MC_BUILDING) std_bld = bld_is_std(a->bld);
  if (n == 0) return PGW_OK;
  // the EV walk split over kEvGroups waves (k_mc_step) where the blocks are at
  // most one per CU anyway: an 11-wave block of 168 VGPRs fits once per CU,
  // where 4-wave blocks fit 3 times
  bool has_ev = false;
  for (int c = 0; c < a->n_comp; ++c) has_ev = has_ev || a->comp[c].kind == PGW_MC_EV;
  const int64_t blocks = (n + 63) / 64;
  const int force = g_mc_ev_split.load(std::memory_order_relaxed);
  // ... and where the walk has more than one chunk: a one-chunk step is one
  // group anyway and the split's barrier and LDS traffic only cost (C3's median
  // step).  The clocked launch (graph replay) cannot see the step: split always.
  int chunks = 2;
  if (has_ev && !a->clock) {
    chunks = 0;
    for (int w = 0; w < a->ev_step.n_words; ++w)
      chunks += (__builtin_popcountll(a->ev_step.scan[w]) + kEvChunk - 1) / kEvChunk;
  }
  const bool split = has_ev && (force >= 0 ? force == 1 : blocks <= 256 && chunks >= 2);
  const dim3 grid((unsigned)blocks), block(64u * (unsigned)(a->n_comp + (split ? kEvGroups - 1 : 0)));
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, block, 0, (hipStream_t)stream, *a, d, n); };
  if (g_mc_trace_on.load() && !a->clock && std::is_same<Args, pgw_mc_step_args>::value)
    std_bld ? go(k_mc_step<Args, true, false, true>) : go(k_mc_step<Args, false, false, true>);
  else if (std_bld)
    a->clock ? go(k_mc_step<Args, true, true>) : go(k_mc_step<Args, true, false>);
  else
    a->clock ? go(k_mc_step<Args, false, true>) : go(k_mc_step<Args, false, false>);
  return check_launch("k_mc_step");
}

extern "C" {

int32_t pgw_mc_agent_step(const pgw_mc_step_args* a, int64_t n, void* stream) {
  return mc_agent_step(a, n, stream);
}

int32_t pgw_mc_agent_step_f32(const pgw_mc_step_args_f32* a, int64_t n, void* stream) {
  return mc_agent_step(a, n, stream);
}

int32_t pgw_ma_step(const pgw_ma_step_args* a, const pgw_pf_params* pf, const pgw_pf_tables* pft,
                    int64_t n, double* v_out, int32_t* iters, void* stream) {
  PGW_REQUIRE(a && n >= 0 && a->n_comp >= 1 && a->n_comp <= PGW_MA_MAX_SLOTS, "pgw_ma_step: bad args");
  PGW_REQUIRE(a->n_agents >= 1 && a->n_agents <= PGW_MAX_AGENTS, "pgw_ma_step: bad n_agents");
  PGW_REQUIRE(a->n_bus >= 0 && a->n_bus <= PGW_PF_MAX_CTRL && (a->n_bus == 0 || a->bus_p),
              "pgw_ma_step: bad n_bus / bus_p");
  int once = 0, pvs = 0, next = 0;
  for (int g = 0; g < a->n_agents; ++g) {
    PGW_REQUIRE(a->agent_first[g] == next && a->agent_count[g] >= 1, "pgw_ma_step: agent %d slots", g);
    next += a->agent_count[g];
    PGW_REQUIRE(a->agent_bus[g] >= -1 && a->agent_bus[g] < a->n_bus, "pgw_ma_step: agent %d bus", g);
    PGW_REQUIRE(!a->agent_sum[g] || (a->agent_real_power[g] && a->agent_reward[g]),
                "pgw_ma_step: agent %d outputs", g);
    PGW_REQUIRE(a->agent_sum[g] || a->agent_count[g] == 1, "pgw_ma_step: agent %d: one slot unless summed", g);
    for (int c = a->agent_first[g]; c < next && c < a->n_comp; ++c)
      PGW_REQUIRE(a->slot_agent[c] == g, "pgw_ma_step: slot %d agent", c);
  }
  PGW_REQUIRE(next == a->n_comp, "pgw_ma_step: agents cover %d of %d slots", next, a->n_comp);
  PGW_REQUIRE(a->n_waves >= 1 && a->n_waves <= a->n_comp, "pgw_ma_step: bad n_waves");
  int listed = 0, wnext = 0;
  for (int w = 0; w < a->n_waves; ++w) {
    PGW_REQUIRE(a->wave_first[w] == wnext && a->wave_count[w] >= 1, "pgw_ma_step: wave %d slots", w);
    wnext += a->wave_count[w];
  }
  PGW_REQUIRE(wnext == a->n_comp, "pgw_ma_step: waves list %d of %d slots", wnext, a->n_comp);
  for (int i = 0; i < a->n_comp; ++i) {
    const int c = a->wave_slot[i];
    PGW_REQUIRE(c >= 0 && c < a->n_comp && !(listed & (1 << c)), "pgw_ma_step: wave_slot %d", i);
    listed |= 1 << c;
  }
  for (int w = 0; w < a->n_waves; ++w)          // (every index below is now < n_comp)
    for (int i = 0; i < a->wave_count[w]; ++i) {
      const int k = a->comp[a->wave_slot[a->wave_first[w] + i]].kind;
      PGW_REQUIRE(a->wave_count[w] == 1 || k == PGW_MC_PV || k == PGW_MC_STORAGE,
                  "pgw_ma_step: a building or EV slot needs a wave of its own");
    }
  // no building: the STD instantiation (its building branch never runs)
  bool std_bld = true;
  for (int c = 0; c < a->n_comp; ++c) {
    const pgw_mc_component& C = a->comp[c];
    PGW_REQUIRE(C.kind >= 0 && C.kind <= 3, "pgw_ma_step: slot %d kind", c);
    PGW_REQUIRE(C.action.ptr && C.obs.ptr && C.real_power, "pgw_ma_step: slot %d buffers", c);
    if (C.kind == PGW_MC_PV) {
      const bool two = a->slot_pv2[c] != 0;
      PGW_REQUIRE(!(pvs & (two ? 2 : 1)), "pgw_ma_step: PV parameter set %d used twice", two ? 2 : 1);
      pvs |= two ? 2 : 1;
      const pgw_pv_params& p = two ? a->pv2 : a->pv;
      const double* vmin = two ? a->pv2_min_voltage : a->pv_min_voltage;
      PGW_REQUIRE(!p.grid_aware || vmin, "pgw_ma_step: slot %d min_voltage", c);
      PGW_REQUIRE(!a->slot_reward[c] || vmin, "pgw_ma_step: slot %d band reward needs min_voltage", c);
    } else {
      PGW_REQUIRE(!(once & (1 << C.kind)), "pgw_ma_step: one building / storage / EV component at most");
      once |= 1 << C.kind;
      PGW_REQUIRE(!a->slot_reward[c], "pgw_ma_step: slot %d: band reward on a PV only", c);
    }
    if (C.kind == PGW_MC_BUILDING) {
      PGW_REQUIRE(a->bld_x && a->bld_reward_state && a->bld.n_obs <= PGW_BLD_MAX_OBS,
                  "pgw_ma_step: building buffers");
      std_bld = bld_is_std(a->bld);
    }
    if (C.kind == PGW_MC_STORAGE) PGW_REQUIRE(a->bat_soc, "pgw_ma_step: storage buffers");
    if (C.kind == PGW_MC_EV)
      PGW_REQUIRE(a->ev_endp && a->ev_req && a->ev_charging && a->ev_reward &&
                  a->ev_step.n_words <= PGW_EV_MAX_WORDS && !a->ev_step.env_start == !a->ev_step.env_endp &&
                  (!a->ev_step.env_start || !a->ev_step.tl_rcp), "pgw_ma_step: EV buffers");
  }
  if (pf) PGW_REQUIRE(pft && pf->n_ctrl == a->n_bus, "pgw_ma_step: pf n_ctrl %d != n_bus %d",
                      pf ? pf->n_ctrl : 0, a->n_bus);
  if (n == 0) return PGW_OK;
  const BldDerived d = make_bld_derived(a->bld);
  const dim3 grid((unsigned)((n + 63) / 64)), block(64u * (unsigned)a->n_waves);
  hipStream_t st = (hipStream_t)stream;
  if (g_mc_trace_on.load())
    std_bld ? launch_timed(PGW_T_MA_STEP, k_ma_step<true, true>, grid, block, st, *a, d, n)
            : launch_timed(PGW_T_MA_STEP, k_ma_step<false, true>, grid, block, st, *a, d, n);
  else if (std_bld)
    launch_timed(PGW_T_MA_STEP, k_ma_step<true>, grid, block, st, *a, d, n);
  else
    launch_timed(PGW_T_MA_STEP, k_ma_step<false>, grid, block, st, *a, d, n);
  const int32_t rc = check_launch("k_ma_step");
  if (rc || !pf) return rc;
  return pgw_pf_solve(pf, pft, n, a->n_bus ? a->bus_p : nullptr, nullptr, v_out, iters, stream);
}

int32_t pgw_agent_reduce(const pgw_reduce_args* a, int64_t n, double* real_power, double* reward,
                         void* stream) {
  PGW_REQUIRE(a && a->n_comp >= 0 && a->n_comp <= PGW_MAX_COMP, "pgw_agent_reduce: bad args");
  PGW_LAUNCH(k_agent_reduce, n, stream, *a, n, real_power, reward);
}

}  // extern "C"
