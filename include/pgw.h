/*
 * pgw.h -- C ABI of libpgw, the MI355X (gfx950) step engine for
 * PowerGridworld-style environments.
 *
 * Boundary rules:
 *   - every array argument is a DEVICE pointer owned by the caller (PyTorch-ROCm
 *     tensors); the library never allocates on the step path;
 *   - state is struct-of-arrays, env index fastest: field f of env e lives at
 *     ptr[f * n + e];
 *   - small per-call parameters are passed as HOST pointers to POD structs and
 *     copied by value into the kernel arguments (so calls are hipGraph-capturable
 *     and reentrant: the library holds no device state);
 *   - calls are asynchronous on `stream` (a hipStream_t, NULL = default stream);
 *   - return 0 on success, < 0 on error (pgw_last_error() gives the message);
 *     no C++ exception crosses the ABI.
 *
 * Each entry point cites the reference interface it replaces
 * (paths relative to lmchion/PowerGridworld).
 */
#ifndef PGW_H_
#define PGW_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PGW_ABI_VERSION 31

#define PGW_OK 0
#define PGW_ERR_ARG (-1)
#define PGW_ERR_HIP (-2)

/* Version of this header the library was built from. */
int32_t pgw_abi_version(void);
/* Message of the last error on the calling thread ("" if none). */
const char* pgw_last_error(void);

/* sizeof() of every ABI struct, in the order pgw_mat, battery_params, pv_params,
 * building_params, building_exo, building_ext, ev_params, ev_step_info,
 * reduce_args, pf_params, pf_tables, feeder_elem, coord_params, coord_buffers,
 * coord_step_info, pred_meta, hs_params, hs_step_info, hs_buffers,
 * mc_step_args, matf, coord_buffers_f32, ma_step_args, pfg_elem, pfg_params,
 * pfg_tables, reg_params, mc_step_dyn, pf_od, mc_step_args_f32 -- lets a
 * binding verify its layouts.  Writes min(n, PGW_N_STRUCT_SIZES) values,
 * returns PGW_N_STRUCT_SIZES. */
#define PGW_N_STRUCT_SIZES 30
int32_t pgw_struct_sizes(int64_t* out, int32_t n);

/* A [n_envs x dim] fp64 matrix in device memory: element (e, j) at
 * ptr[e * s_env + j * s_dim].  Used for actions (read) and observations
 * (written), so callers can hand over row-major [N, dim] policy tensors or
 * env-minor [dim, N] buffers without a copy. */
typedef struct pgw_mat {
  double* ptr;
  int64_t s_env;
  int64_t s_dim;
} pgw_mat;

/* fp32 variant of pgw_mat, for the *_f32 entries.  The f32 entries store state,
 * actions and outputs as fp32 (half the HBM bytes) but compute in fp64
 * registers: each value is widened on load and rounded once at its store, so
 * the only deviation from the fp64 path is the storage rounding (~6e-8 rel per
 * step; the north-star bound for fp32 is 1e-3 rel). */
typedef struct pgw_matf {
  float* ptr;
  int64_t s_env;
  int64_t s_dim;
} pgw_matf;

/* PGW_OOB -- out-of-bounds actions.  The reference's to_raw warns when a
 * rescaled action leaves [-1 - 1e-4, 1 + 1e-4] (or is NaN) and clips it
 * (gridworld/utils.py:35-40).  The kernels clip the same way; when a
 * component's params carry a non-NULL `oob` (device uint64), every to_raw
 * call the reference would have warned on -- one per (env, component, step),
 * whatever the number of offending elements -- adds 1 to it (a vector atomic,
 * only on that rare path).  The caller reads it whenever it likes. */
#define PGW_OOB_EPS 1e-4

/* ------------------------------------------------------------------------
 * Energy storage.  Replaces EnergyStorageEnv.reset/step/get_obs
 * (gridworld/agents/energy_storage/energy_storage_env.py:72-178).
 * ---------------------------------------------------------------------- */
typedef struct pgw_battery_params {
  double soc_min, soc_max;   /* storage_range            (:23)  */
  double eta_c, eta_d;       /* charge/discharge eff.    (:26-27) */
  double max_power;          /* kW                       (:28)  */
  double dt_h;               /* control_timedelta in h   (:49)  */
  int32_t rescale;           /* rescale_spaces           (:31)  */
  int32_t sampled_init;      /* reset only: 1 = init_soc was drawn (truncnorm, :80-84)
                                and is taken as is; 0 = a given init_storage, clipped
                                to storage_range (:86-95).  The step ignores it. */
  uint64_t* oob;             /* nullable device counter, see PGW_OOB below */
} pgw_battery_params;

/* soc[e] = init_soc[e], clipped to [soc_min, soc_max] unless p->sampled_init;
 * obs = SoC (scaled). (:72-97) */
int32_t pgw_battery_reset(const pgw_battery_params* p, int64_t n, const double* init_soc,
                          double* soc, pgw_mat obs, void* stream);
/* One control step: to_raw, validate_power, SoC update, real_power = -power.
 * Reward is identically 0 (:159-164).  (:100-157) */
int32_t pgw_battery_step(const pgw_battery_params* p, int64_t n, pgw_mat action,
                         double* soc, pgw_mat obs, double* real_power, void* stream);
/* fp32-storage variants of the two entries above (fp64 arithmetic). */
int32_t pgw_battery_reset_f32(const pgw_battery_params* p, int64_t n, const float* init_soc,
                              float* soc, pgw_matf obs, void* stream);
int32_t pgw_battery_step_f32(const pgw_battery_params* p, int64_t n, pgw_matf action,
                             float* soc, pgw_matf obs, float* real_power, void* stream);

/* ------------------------------------------------------------------------
 * PV curtailment.  Replaces PVEnv.get_obs/step
 * (gridworld/agents/pv/pv_profile_env.py:102-148).
 * ---------------------------------------------------------------------- */
typedef struct pgw_pv_params {
  double obs_low, obs_high;     /* (-max(data), 0)           (:86-96) */
  double vmin_low, vmin_high;   /* (0.9, 1.1) when grid_aware */
  int32_t rescale, grid_aware;
  uint64_t* oob;                /* nullable device counter, see PGW_OOB */
} pgw_pv_params;

/* obs only (PVEnv.get_obs at the current index); `pmax` = data[index]. */
int32_t pgw_pv_obs(const pgw_pv_params* p, int64_t n, double pmax, const double* min_voltage,
                   pgw_mat obs, void* stream);
/* obs (pre-advance, :143) and real_power = to_raw(a,0,1) * (-pmax) (:144). */
int32_t pgw_pv_step(const pgw_pv_params* p, int64_t n, double pmax, pgw_mat action,
                    const double* min_voltage, pgw_mat obs, double* real_power, void* stream);
/* fp32 storage (obs, action, real power), fp64 arithmetic; min_voltage stays
 * the fp64 power-flow output. */
int32_t pgw_pv_obs_f32(const pgw_pv_params* p, int64_t n, double pmax, const double* min_voltage,
                       pgw_matf obs, void* stream);
int32_t pgw_pv_step_f32(const pgw_pv_params* p, int64_t n, double pmax, pgw_matf action,
                        const double* min_voltage, pgw_matf obs, float* real_power, void* stream);

/* ------------------------------------------------------------------------
 * Five-zone reduced-order building.  Replaces FiveZoneROMEnv.reset/step_/get_obs
 * and FiveZoneROMThermalEnergyEnv.step_reward
 * (gridworld/agents/buildings/five_zone_rom_env.py:147-335,
 *  five_zone_rom_dynamics.py:12-114).
 * ---------------------------------------------------------------------- */
#define PGW_BLD_MAX_OBS 24   /* 15 zone values + 9 scalars */

/* observation variable ids, in the reference's state-dict order (:230-246) */
enum {
  PGW_BV_ZONE_TEMP = 0,        /* + zone (0..4) */
  PGW_BV_UPPER_VIOL = 5,       /* + zone */
  PGW_BV_LOWER_VIOL = 10,      /* + zone */
  PGW_BV_COMFORT_LOWER = 15,
  PGW_BV_COMFORT_UPPER = 16,
  PGW_BV_OUTDOOR_TEMP = 17,
  PGW_BV_P_CONSUMED = 18,
  PGW_BV_TIME_OF_DAY = 19,
  PGW_BV_BUS_VOLTAGE = 20,
  PGW_BV_MIN_VOLTAGE = 21,
  PGW_BV_MAX_VOLTAGE = 22,
  PGW_BV_P_SETPOINT = 23
};

typedef struct pgw_building_params {
  double A[5];           /* ss_A                                   */
  double B[5][4];        /* ss_B rounded to float32 (dynamics.py:51) */
  double K[5];           /* ss_K (filter gain)                     */
  double C[5];           /* ss_C                                   */
  double mean[5];        /* mean_output                            */
  double act_low[6], act_high[6];   /* (:22-26)                    */
  double T_init[5];      /* zone_temp_init (:91)                   */
  double obs_low[PGW_BLD_MAX_OBS], obs_high[PGW_BLD_MAX_OBS];  /* make_obs_space order */
  double alpha;          /* 0.2 (:318)                             */
  int32_t sel[5][4];     /* input_sel_list - 1 (index into u_pos)  */
  int32_t nbr[5][4];     /* neighbors                              */
  int32_t obs_var[PGW_BLD_MAX_OBS];   /* PGW_BV_* per obs slot, state-dict order */
  int32_t n_obs;
  int32_t rescale;
  uint64_t* oob;         /* nullable device counter, see PGW_OOB     */
} pgw_building_params;

/* Exogenous row (shared by all envs, host values) + the obs-time scalars. */
typedef struct pgw_building_exo {
  double T_oa;
  double q_solar[5], q_int[5], q_cool[5];
  double comfort_lb, comfort_ub;
  double time_of_day;    /* time_index / max_episode_steps */
  double pad_;
} pgw_building_exo;

/* External obs inputs (device [n] arrays); NULL selects the reference default
 * (bus/min/max voltage 1.0 -- or bus_voltage when given --, p_setpoint +inf). */
typedef struct pgw_building_ext {
  const double* bus_voltage;
  const double* min_voltage;
  const double* max_voltage;
  const double* p_setpoint;
} pgw_building_ext;

/* reset: u from q_cool at row 0, two filter updates, obs at row 0.  x (5 x n,
 * zone-major) is updated IN PLACE: the Kalman state persists across resets as in
 * the reference (:147-180).  p_consumed := 0; reward_state := reward of the reset
 * state (what the first standalone step returns). */
int32_t pgw_building_reset(const pgw_building_params* p, const pgw_building_exo* ex0, int64_t n,
                           double* x, double* p_consumed, double* reward_state,
                           pgw_building_ext ext, pgw_mat obs, void* stream);
/* step: to_raw, dynamics with row `ex_t`, p_consumed, advance, obs with row
 * `ex_next`.  reward_out gets the PREVIOUS state's reward when lagged != 0
 * (standalone env, :215) or the fresh reward otherwise (MultiComponentEnv,
 * base.py:137); reward_state always ends holding the fresh reward. */
int32_t pgw_building_step(const pgw_building_params* p, const pgw_building_exo* ex_t,
                          const pgw_building_exo* ex_next, int64_t n, pgw_mat action, double* x,
                          double* p_consumed, double* reward_out, double* reward_state,
                          int32_t lagged, pgw_building_ext ext, pgw_mat obs, void* stream);
/* fp32 storage of the state (x, p_consumed, rewards), obs and actions; fp64
 * arithmetic, each value rounded once at its store. */
int32_t pgw_building_reset_f32(const pgw_building_params* p, const pgw_building_exo* ex0, int64_t n,
                               float* x, float* p_consumed, float* reward_state,
                               pgw_building_ext ext, pgw_matf obs, void* stream);
int32_t pgw_building_step_f32(const pgw_building_params* p, const pgw_building_exo* ex_t,
                              const pgw_building_exo* ex_next, int64_t n, pgw_matf action, float* x,
                              float* p_consumed, float* reward_out, float* reward_state,
                              int32_t lagged, pgw_building_ext ext, pgw_matf obs, void* stream);

/* ------------------------------------------------------------------------
 * EV charging station.  Replaces EVChargingEnv.reset/step/step_reward
 * (gridworld/agents/vehicles/ev_charging_env.py:135-264).
 * ---------------------------------------------------------------------- */
#define PGW_EV_MAX_WORDS 16   /* up to 1024 vehicles */

typedef struct pgw_ev_params {
  double rate;           /* max_charge_rate_kw       */
  double hours_per_step; /* minutes_per_step / 60.   */
  double mult;           /* vehicle_multiplier       */
  double u_pen, p_pen, thr, reward_scale;
  double obs_low[6], obs_high[6];
  int32_t n_vehicles, rescale;
  uint64_t* oob;         /* nullable device counter, see PGW_OOB */
} pgw_ev_params;

/* Per-step schedule, shared by all envs (time is lockstep): bit v of `window`
 * = vehicle v parked (start <= time <= end_park), of `scan` = parked now or at the
 * previous step. */
typedef struct pgw_ev_step_info {
  double time;           /* minutes, before the step's advance        */
  double next_time;      /* simulation_times[time_index + 1]          */
  double action_default; /* raw action used when action.ptr == NULL (reset step) */
  /* Optional (device, NULL = computed in the kernel): per vehicle v,
   * tl_rcp[2v] = (end_park[v] - time) / 60 (time left in hours, the
   * reference's expression, :199) and tl_rcp[2v+1] = 1 / tl_rcp[2v], so the
   * per-vehicle division by it is exact_div (bit-identical, no IEEE divide). */
  const double* tl_rcp;
  /* Optional (device, NULL = the shared schedule above): per-env vehicle
   * tables, V x n, for randomize=True (each env drew its own vehicle subset,
   * ev_charging_env.py:154-156).  env_start = floor(rounded start_time_min),
   * env_endp = rounded end_time_park_min.  Then `window` is ignored (parked =
   * env_start <= time <= floor(env_endp), per env), `scan` must hold all
   * n_vehicles bits and tl_rcp must be NULL (time left is divided in IEEE). */
  const double* env_start;
  const double* env_endp;
  int32_t n_words, pad_;
  uint64_t window[PGW_EV_MAX_WORDS];
  uint64_t scan[PGW_EV_MAX_WORDS];
} pgw_ev_step_info;

/* req (V x n) := req0 (V) broadcast; charging bits := 0. */
int32_t pgw_ev_reset(const pgw_ev_params* p, int64_t n, const double* req0, double* req,
                     uint64_t* charging, void* stream);
/* randomize=True reset (:154-156): req (V x n) := req0_env (V x n, each env's
 * sampled vehicles' energy_required_kwh * multiplier); charging bits := 0. */
int32_t pgw_ev_reset_tables(const pgw_ev_params* p, int64_t n, const double* req0_env, double* req,
                            uint64_t* charging, void* stream);
/* One step (reset's action-less step when action.ptr == NULL).  endp = rounded
 * end_time_park_min (V).  Writes obs (6), real_power, reward. */
int32_t pgw_ev_step(const pgw_ev_params* p, const pgw_ev_step_info* s, int64_t n, pgw_mat action,
                    const double* endp, double* req, uint64_t* charging, pgw_mat obs,
                    double* real_power, double* reward, void* stream);
/* fp32 storage of the requirements, obs, actions, real power and reward;
 * fp64 arithmetic (the parked masks, the vehicle tables and req0 as above). */
int32_t pgw_ev_reset_f32(const pgw_ev_params* p, int64_t n, const double* req0, float* req,
                         uint64_t* charging, void* stream);
int32_t pgw_ev_reset_tables_f32(const pgw_ev_params* p, int64_t n, const double* req0_env, float* req,
                                uint64_t* charging, void* stream);
int32_t pgw_ev_step_f32(const pgw_ev_params* p, const pgw_ev_step_info* s, int64_t n, pgw_matf action,
                        const double* endp, float* req, uint64_t* charging, pgw_matf obs,
                        float* real_power, float* reward, void* stream);
/* Doubles per env row of the env-major requirement layout for n_vehicles. */
int32_t pgw_ev_row(int32_t n_vehicles);
/* pgw_ev_step on env-major requirements: req (n x pgw_ev_row(V)), per-env
 * tables likewise; lanes over vehicles, a wave per 1-4 envs. */
int32_t pgw_ev_step_lanes(const pgw_ev_params* p, const pgw_ev_step_info* s, int64_t n, pgw_mat action,
                          const double* endp, double* req, uint64_t* charging, pgw_mat obs,
                          double* real_power, double* reward, void* stream);

/* ------------------------------------------------------------------------
 * MultiComponentEnv reduction (gridworld/base.py:125-156): real_power and
 * reward summed in component order starting from 0.
 * ---------------------------------------------------------------------- */
#define PGW_MAX_COMP 8
typedef struct pgw_reduce_args {
  const double* real_power[PGW_MAX_COMP];  /* NULL = contributes 0 */
  const double* reward[PGW_MAX_COMP];      /* NULL = contributes 0 */
  int32_t n_comp, pad_;
} pgw_reduce_args;
int32_t pgw_agent_reduce(const pgw_reduce_args* a, int64_t n, double* real_power, double* reward,
                         void* stream);

/* ------------------------------------------------------------------------
 * Distribution power flow.  Replaces OpenDSSSolver.calculate_power_flow +
 * get_bus_voltages (gridworld/distribution_system/opendss.py:80-165); the
 * per-env snap solve is a fixed-point current-injection iteration on the
 * load-element voltages  U = U0 + W f(U)  (see DESIGN.md).
 * ---------------------------------------------------------------------- */
#define PGW_PF_MAX_M 16     /* load phase elements (IEEE-13: 14) */
#define PGW_PF_MAX_CTRL 8   /* controllable loads     */

typedef struct pgw_pf_params {
  double vbase[PGW_PF_MAX_M];       /* element base voltage (V)               */
  double vmin[PGW_PF_MAX_M], vmax[PGW_PF_MAX_M], vlow[PGW_PF_MAX_M];  /* pu   */
  double nph[PGW_PF_MAX_M];          /* phases of the element's load           */
  double base_kw[PGW_PF_MAX_M];     /* the element's LOAD total kW this step  */
  double base_kvar[PGW_PF_MAX_M];   /*   (loadshape x base x rescale)         */
  double tol;                       /* max |dU|/vbase convergence tolerance   */
  double pred_x0, pred_h;           /* predictor grid: kW of point j = x0 + j h */
  int32_t elem_ctrl[PGW_PF_MAX_M];  /* controllable-load slot of the element, -1 none */
  int32_t m;                        /* element count, = pgw_pf_padded_m(true m) */
  int32_t n_ctrl, n_out, max_iter;
  int32_t pred_n;                   /* predictor grid points (>= 3 to use U_pred) */
} pgw_pf_params;

/* Predictor stencil metadata of one grid segment (see pgw_pf_tables.U_pred_meta). */
typedef struct pgw_pred_meta {
  double tstar;           /* switch position inside the segment, in [0, 1] */
  int32_t left, right;    /* record (stencil centre) used left / right of it */
} pgw_pred_meta;

/* Device tables.  `block` is the wave-uniform operand block the solve streams
 * through the scalar cache every iteration; build it on the host with
 * pgw_pf_pack from W = -C Z C^T and U0 = C V0 (pgw_pf_reduce) and copy it to
 * the device once per feeder / output-node set. */
typedef struct pgw_pf_tables {
  const double* block;  /* pgw_pf_pack_size(m) doubles (device)           */
  /* Output rows in per unit, against the scaled element currents I'_k = I_k vb_k:
   * G: n_out x m complex, G_ok / (vb_k vb_o) with G = -(Z C^T)[output nodes];
   * V0: n_out complex, V0_o / vb_o (no-load node voltage). */
  const double* G;
  const double* V0;
  /* Optional initial guess (n_ctrl == 1 only): pred_n predictor records
   * (pgw_pf_pred_pack) of the grid solutions at controllable load
   * x_j = pred_x0 + j pred_h for this step's base loads; each env starts from
   * the quadratic of a record near its own controllable kW instead of from U0.
   * The converged result is the same fixed point (to tol); only the iteration
   * count drops.  NULL = cold start from U0. */
  const double* U_pred;
  /* Optional stencil choice per grid segment (pgw_pf_pred_meta, pred_n - 1
   * entries): an env in segment j at fractional position t uses the record
   * centred at meta[j].left if t < meta[j].tstar, else at meta[j].right -- so
   * its quadratic never straddles a load-band switch (an element crossing
   * vlow/vmin/vmax, where the solution is not smooth in the controllable kW).
   * NULL = the record nearest the env. */
  const struct pgw_pred_meta* U_pred_meta;
  /* Optional per-env initial guess, n x m complex element voltages in per unit
   * of each element's vbase (env-major); overrides U_pred.  NULL = none. */
  const double* U_init;
  /* Optional output: converged element voltages, n x m complex in per unit of
   * each element's vbase (env-major). */
  double* U_out;
  /* Optional output: per env, the band of every element in 2 bits (element k
   * in bits 2k..2k+1: 0 |u| <= vlow, 1 <= vmin, 2 <= vmax, 3 above). */
  int32_t* sig_out;
  /* Optional per-env multiplier of base_kw / base_kvar (n doubles): solves
   * several load levels (e.g. the loadshape hours of an episode) in one launch.
   * NULL = 1. */
  const double* load_scale;
  /* Optional outputs of pgw_pf_solve (n doubles each): the minimum / maximum
   * over the n_out output rows, taken in row order as Python's min()/max() do
   * over the voltage dict (multiagent_env.py:107-113).  NULL = not written. */
  double* v_min_out;
  double* v_max_out;
  /* OpenDSS's own snap solve on the fast kernels (HOST pointer, NULL = the
   * exact fixed point): see pgw_pf_od below. */
  const struct pgw_pf_od* od;
} pgw_pf_tables;

/* OpenDSS's snap solve (opendss.py:134 `Solve mode=snap`; Solution.pas
 * SolveSnap -> DoNormalSolution, restated in oracle/pf_oracle.py
 * Feeder.snap_opendss) on pgw_pf_solve / pgw_coord_step's one-lane-per-env
 * kernels, for feeders of the fast shape (m = 14 constant-PQ elements, one
 * voltage band, at most one controllable slot): the packed block holds the
 * iteration matrix of Y + every load's nominal Yeq (W'' of that Y, u0 = the
 * direct solution C Y^-1 I_src); element k's current is I'_k = (conj(S_k) g -
 * y0'_k) u_k, y0' = the per-phase conj(S) whose Yeq sits in Y; the solve stops
 * at the first iteration >= min_iter whose largest node-voltage magnitude
 * change (pu of the node base) is <= tol, or at max_iter (-iterations).
 *
 * Node magnitudes: an element from a node to ground gives that node's |V| =
 * |u_k| elem_scale[k] (0 = the element is not a node).  The other nodes are
 * check rows (rows_V0 / rows_G: V = V0 + G I', pu of the node base against the
 * scaled currents, the layout of pgw_pf_tables.G): rows [0, n_rep) are
 * evaluated when a test needs them; rows [n_rep, n_rows) are bounded instead,
 * members (electrically next to a row or an element node: |G_j - G_r| <= gamma
 * per element, |V0_j - V0_r| <= eps) and source-side nodes (|G_j| <= gsrc per
 * element), with gmax >= |G_r| per element of every row and element node; when
 * a bound cannot decide an env's test, its wave evaluates the bounded rows too
 * (that iteration), so the stopping iteration is always the exact rule's.  The
 * rows are evaluated only in iterations where some env of the wave has no
 * element node whose change is surely above tol (min_iter >= 2).  A wave with
 * at most sparse_envs envs to test evaluates their rows one env at a time
 * (one lane per row) instead of as every lane's row groups -- same values,
 * bit for bit; sparse_envs 0 = the default (4), < 0 = never.
 *
 * start (device, this step's hour): the first iteration in closed form -- from
 * the direct solution the currents are affine in the env's controllable
 * (P, Q): u_1 = u1b + P u1P + Q u1Q and J_1 = J1b + P J1P + Q J1Q; u1b, u1P,
 * u1Q, J1b, J1P, J1Q (m complex each).
 *
 * resp (device, this step's hour; NULL = every env runs the snap solve): the
 * RESPONSE TABLE of the hour's snap solve.  With one controllable slot and
 * Q = 0 the whole stopped solve -- its iteration count k* and the accepted
 * iteration's compensation currents J' = I'(u_{k*-1}), from which every node
 * voltage follows as V0 + G J' -- is a function of the env's kW P alone,
 * smooth between breakpoints where k* changes or an element's |u| crosses its
 * band limit in one of the iterates.  The table holds it per piece as a
 * quadratic in P; OpenDSSSolver builds it with pgw_pf_od_probe (the same snap
 * solve at chosen P: the breakpoints by bisection of its signature, three fit
 * points per piece, two check points whose error bounds the fit).  Segment j of
 * the grid resp_x0 + j / resp_inv_h (j < resp_nseg) has its first piece at
 * record j, further pieces chained by `next`; an env whose P lies in no piece
 * (a breakpoint's bracket, outside the grid, Q != 0, a piece marked
 * unfittable) runs the snap solve instead.  Every served interval is
 * certified (OpenDSSSolver._od_response, od_certify.py): Taylor-model bounds
 * of the iterates over the whole interval prove each element's band in each
 * iterate and each stopping test's outcome constant there (margins >= 1e-12,
 * far above the kernels' rounding), and a piece that cannot be proven whole
 * serves only its longest certified run ([0] lo / [1] hi narrowed).  So the
 * table changes no decision: results differ from the solve only by the fit
 * error (checked <= the builder's tolerance at the check points).  Record
 * layout: PGW_OD_REC. */
#define PGW_PF_OD_MAX_ROWS 28
/* Response-table record of m elements, doubles: [0] lo, [1] hi (kW; the piece
 * covers lo <= P <= hi), [2] xc, [3] inv_hw (t = (P - xc) inv_hw), [4] two
 * int32 (iterations k*, 0 = no fit; next record of the segment, -1 = none),
 * [5] reserved, then c0, c1, c2 (2 m each, re / im per element):
 * J'_k(t) = c0_k + t (c1_k + t c2_k). */
#define PGW_OD_REC_HEAD 6
#define PGW_OD_REC(m) (PGW_OD_REC_HEAD + 6 * (m))
/* Node records (resp_v, optional): one per response record, same index, 12
 * doubles: the record's header [0..5] copied, then the fitted complex voltage
 * (pu) of one node, V(t) = v0 + t (v1 + t v2), [6..11] = v0, v1, v2 (re, im):
 * V0_node + G_node J'(t) composed on the host.  Output row resp_v_row (the
 * controllable load's node) is then read from it for every env the table
 * serves, and a solve whose only output is that row reads 96 bytes per env
 * instead of the 720-byte record. */
#define PGW_OD_VREC 12
/* Extrema rows (resp_rows, ABI 29; 0 = every row): with v_out NULL and the
 * extrema wanted (pgw_pf_tables.v_min_out / v_max_out), bit r set for output
 * row r (1 <= r < 64) that can be the minimum or the maximum |V| of an env
 * the hour's table serves -- proved on the host from the records' quadratics
 * (interval bounds of every row's |V|^2 over every served piece, with a
 * margin far above rounding): a wave whose envs are all served evaluates
 * only those rows (and row 0), which leaves every extremum's value unchanged;
 * a wave with an env solved in full evaluates every row. */
typedef struct pgw_pf_od {
  double tol;                        /* 1e-4 (ConvergenceTolerance)            */
  double y0r[PGW_PF_MAX_M], y0i[PGW_PF_MAX_M];   /* y0' per element (W, -var) */
  double elem_scale[PGW_PF_MAX_M];   /* node |V| pu = |u_k| * scale; 0 = none   */
  double gamma, eps, gmax, gsrc;     /* check-row bound constants (above)      */
  int32_t min_iter;                  /* 2 (MinIterations); >= 2                */
  int32_t n_rep, n_rows;
  int32_t sparse_envs;               /* 0 = default (4); < 0 never; <= 64     */
  const double* rows_V0;             /* n_rows complex (device)                */
  const double* rows_G;              /* n_rows x m complex (device)            */
  const double* start;               /* 12 m doubles (device)                  */
  const double* resp;                /* response table records (device) or NULL */
  double resp_x0, resp_h;            /* grid origin and step (kW)               */
  int32_t resp_nseg;                 /* grid segments (primary records)         */
  int32_t resp_v_row;                /* output row of the node records; < 0 none */
  const double* resp_v;              /* node records (PGW_OD_VREC each) or NULL */
  uint64_t resp_rows;                /* extrema rows of served envs; 0 = all    */
  /* Row records (or NULL): per response record, PGW_OD_REC_HEAD header
   * doubles (a bitwise copy of the response record's) then, for the k-th set
   * bit r of resp_q_rows (ascending; output rows < 64), the squared magnitude
   * of output row r as a quartic in the record's t: a0..a4 at
   * [PGW_OD_REC_HEAD + 5 k ..], |V_r|^2 = a0 + t (a1 + t (a2 + t (a3 + t a4))).
   * A served env takes every listed row from them on every path.  resp_q_k =
   * popcount(resp_q_rows); records resp_q_stride doubles apart. */
  const double* resp_q;
  uint64_t resp_q_rows;
  int32_t resp_q_stride, resp_q_k;
} pgw_pf_od;

/* Element k draws S_k = ((base_kw[k] + ctrl_p[elem_ctrl[k]]) * 1000 / nph[k]) + j(...kvar)
 * (opendss.py:107-129 then OpenDSS's per-phase WNominal).
 * ctrl_p / ctrl_q: n_ctrl x n (kW / kvar, NULL = 0).  v_out: n_out x n (pu); NULL
 * when only the extrema (pgw_pf_tables.v_min_out / v_max_out) are wanted.
 * iters: n (int32, nullable) iteration count per env; -count when the env stopped
 * at max_iter without passing the convergence test. */
int32_t pgw_pf_solve(const pgw_pf_params* p, const pgw_pf_tables* t, int64_t n,
                     const double* ctrl_p, const double* ctrl_q, double* v_out,
                     int32_t* iters, void* stream);
/* fp32-storage variant: ctrl_p / ctrl_q / v_out float, widened
 * on load and rounded once on store; the solve itself is the fp64 one (same
 * kernels, same iteration counts), and the pgw_pf_tables outputs (extrema,
 * element voltages) stay double. */
int32_t pgw_pf_solve_f32(const pgw_pf_params* p, const pgw_pf_tables* t, int64_t n,
                         const float* ctrl_p, const float* ctrl_q, float* v_out,
                         int32_t* iters, void* stream);

/* Response-table builder (OpenDSSSolver._od_response): the snap solve of
 * pgw_pf_od at n lanes, lane e at controllable kW P[e] (Q = 0) in hour
 * e / lanes_per_hour (a multiple of 256): hour h uses p_hours[h] (its base
 * loads) and the first-iteration table start_h + 12 m h; t->od holds the
 * hour-independent rest (its start and resp are ignored).  Writes per lane the
 * accepted iteration's currents J_out[e][k] (m complex, the pgw_pf_od.resp
 * quantity), the iteration count it_out[e] (as pgw_pf_solve's iters) and
 * sig_out[e], a 64-bit hash of the count and the band states of every iterate
 * whose currents the solve formed -- equal signatures: the same piece.
 * args_buf: device scratch of pgw_pf_od_probe_args_size(n_hours) bytes. */
int64_t pgw_pf_od_probe_args_size(int32_t n_hours);
int32_t pgw_pf_od_probe(const pgw_pf_params* p_hours, int32_t n_hours, const pgw_pf_tables* t,
                        const double* start_h, int32_t lanes_per_hour, int64_t n, const double* P,
                        double* J_out, uint64_t* sig_out, int32_t* it_out, void* args_buf, void* stream);

/* Pieces -> response records (device).  Piece i: fit points a < mid < b whose
 * currents are J[ia], J[im], J[ib] (m complex each; idx3[3 i ..]), its
 * covered range [lo, hi] and xc, inv_hw (meta[4 i ..]), its iteration count
 * and next record (inext[2 i ..]), written to record rec[i] of `out`:
 * c0 = J(mid), c1 = (J(b) - J(a)) / 2, c2 = (J(a) + J(b)) / 2 - J(mid) (the
 * quadratic through the three points when mid is the middle). */
int32_t pgw_pf_od_resp_fit(int32_t m, int64_t n_pieces, const double* J, const int32_t* idx3,
                           const double* meta, const int32_t* inext, const int32_t* rec, double* out,
                           void* stream);

/* Fit check: err[i] = max_k |J'_k(P_i) - J[iq_i][k]| / max_k |J[iq_i][k]| for
 * the piece in record rec[i] evaluated at P[i] exactly as the step kernels do. */
int32_t pgw_pf_od_resp_check(int32_t m, int64_t n, const double* recs, const int32_t* rec, const double* P,
                             const double* J, const int32_t* iq, double* err, void* stream);

/* Predictor records from grid solutions (device): U_grid n_tables x n_points x m
 * complex (U_out of the grid solve) -> rec, n_tables x n_points records of
 * 32 m bytes: u_j (m complex fp64), then d1 = u_{j+1} - u_{j-1} and
 * d2 = u_{j+1} - 2 u_j + u_{j-1} (m complex fp32 each; end points use the
 * neighbouring interior centre's differences).  u(t) = u_j + t d1/2 + t^2 d2/2
 * is the 3-point quadratic centred at j.  16-byte aligned. */
int32_t pgw_pf_pred_pack(const pgw_pf_params* p, int32_t n_tables, int32_t n_points,
                         const double* U_grid, double* rec, void* stream);
/* Stencil metadata for n_tables predictor grids of n_points solutions each
 * (U_grid: n_tables x n_points x m complex, sig: their sig_out) -> meta:
 * n_tables x (n_points - 1).  Uses p's per-element voltage bands.  Device. */
int32_t pgw_pf_pred_meta(const pgw_pf_params* p, int32_t n_tables, int32_t n_points,
                         const double* U_pred, const int32_t* sig, pgw_pred_meta* meta,
                         void* stream);

/* Voltage-band penalty of the heterogeneous scenario's PV farm
 * (gridworld/scenarios/heterogeneous.py:47-52, ThisPVEnv.step_reward):
 * out[e] = -(scale * (min(0, v[e] - lo) + min(0, hi - v[e])))^2. */
int32_t pgw_voltage_band_penalty(int64_t n, const double* v, double lo, double hi, double scale,
                                 double* out, void* stream);

/* Element count the kernels are instantiated for (8, 14 or 16): pad the
 * feeder's m load phase elements to it with inert elements (zero power). */
int32_t pgw_pf_padded_m(int32_t m);
/* Doubles in the packed operand block for padded element count m. */
int64_t pgw_pf_pack_size(int32_t m);
/* Host memory: pack W (m x m complex, row-major; must be complex symmetric),
 * U0 (m complex), the per-element voltage bands of p and output row 0 of the
 * tables (G0: m complex, V0_0: complex -- required if p->n_out > 0) into `out`
 * (pgw_pf_pack_size(p->m) doubles). */
int32_t pgw_pf_pack(const pgw_pf_params* p, const double* W, const double* U0, const double* G0,
                    const double* V0_0, double* out);

/* ------------------------------------------------------------------------
 * General batched power flow: any feeder size (PGW_PFG_MAX_M load phase
 * elements) and two stopping rules.  Replaces the same OpenDSSSolver.
 * calculate_power_flow (opendss.py:80-165) as pgw_pf_solve, for feeders beyond
 * PGW_PF_MAX_M and for OpenDSS's own iteration (opendss.py:134 `Solve
 * mode=snap`):
 *   PGW_PF_EXACT    u <- u0 + W I'(u) from u0 (or U_init) until every element's
 *                   |du| < tol (pu of its base): the fixed point, as pgw_pf_solve;
 *   PGW_PF_OPENDSS  OpenDSS's snap solve (Solution.pas DoNormalSolution): Y holds
 *                   each load's nominal admittance (elem.y0), the iteration starts
 *                   from the direct solution u0 = C Y^-1 I_src, injects the
 *                   compensation current I_load(u) - y0 u, and stops at the first
 *                   iteration >= min_iter whose largest change of a node-voltage
 *                   magnitude over the n_chk check rows (every node, pu of the
 *                   node base) is <= tol, or at max_iter.
 * Per-unit form as pgw_pf_solve: u = U / vb, I' = I vb = (conj(S) g - y0') u with
 * y0' = conj(S_y0) (the per-phase power whose Yeq sits in Y).  Element k draws
 * S_k = ((coef * base_kw) * rescale + ctrl_p[ctrl]) * 1000 / nph (+ j likewise):
 * opendss.py:105-131 then OpenDSS's per-phase WNominal.
 * Layout: a block of 4 waves serves 64 envs (lane = env); element, check and
 * output rows are split over the waves in chunks of 8, and every row is
 * accumulated against the element currents through LDS with its matrix entries
 * as wave-uniform scalar operands.  Matrices are column (element) major with
 * rows padded to a multiple of 8: M[2 (k ld + row) + re/im].
 * ---------------------------------------------------------------------- */
#define PGW_PFG_MAX_M 128     /* load phase elements */
#define PGW_PFG_MAX_CHK 256   /* OpenDSS check rows (nodes) */
/*   PGW_PF_OPENDSS_STEP  the same snap solve with every load's Yeq in Y at the
 *                   STEP's powers (the reading in which the Loads.kW setters
 *                   re-stamp Yprim, H1): y0' = the element's own conj(S); the
 *                   tables hold the hour's reduction (per-hour Yeq) and the
 *                   controllable elements' per-env Yeq change enters as the
 *                   n_reg correction columns (Kreg = (I - D W_cc)^-1 D per env,
 *                   reg_rho = 1), as RegControl taps do. */
enum { PGW_PF_EXACT = 0, PGW_PF_OPENDSS = 1, PGW_PF_OPENDSS_STEP = 2 };

typedef struct pgw_pfg_elem {
  double base_kw, base_kvar;   /* the element's LOAD kW / kvar before loadshape and rescale */
  double nph;                  /* phases of that load                                  */
  double y0r, y0i;             /* OPENDSS: conj(S) per phase (W, -var) of the Yeq in Y; 0 */
  double vlo2, vmn2, vmx2;     /* vlow^2, vmin^2, vmax^2 (pu^2)                         */
  int32_t ctrl;                /* controllable-load slot, -1 none                      */
  /* OpenDSS load model of the element: 1 constant PQ (loadshape-scaled, may be
   * controllable), 3 constant P + constant-Z Q, 4 exponential (exp_p = CVRwatts,
   * exp_q = CVRvars), 5 constant current magnitude, 6 constant P + fixed Q,
   * 7 constant P + fixed-impedance Q, 8 ZIP (zip = Zp Ip Pp Zq Iq Pq, load off
   * below vcut2 = cutoff^2).  Models 3-8 keep base_kw / base_kvar unscaled (the
   * reference re-sets model-1 loads only, opendss.py:71,149). */
  int32_t model;
  double exp_p, exp_q;
  double zip[6];
  double vcut2;
} pgw_pfg_elem;

typedef struct pgw_pfg_params {
  int32_t m;          /* element rows (padded to 8 with inert zero-power elements)   */
  int32_t n_chk;      /* OPENDSS check rows (padded to 8; 0 for EXACT)               */
  int32_t n_out;      /* output rows                                                 */
  int32_t n_ctrl;
  int32_t mode, min_iter, max_iter, pad_;
  double tol;
  double coef, rescale;   /* the step's loadshape coefficient, system_load_rescale_factor */
  /* Regulators under RegControl (per-env taps): n_reg regulator terminal nodes
   * R (padded to 8, <= PGW_PFG_MAX_REG; 0 = none), r_reg of them real.  The
   * solve with taps t is the DSS-tap solve (the tables) corrected exactly
   * (Woodbury): with x = the DSS-tap node voltages at R for the iterate's
   * currents, c = K(t) x (per env, pgw_reg_factor) and every row gains -(Z0 U c)
   * -- as n_reg extra current columns c after the m element columns of W, Gc
   * and G (so those tables have m + n_reg columns). */
  int32_t n_reg, r_reg;
} pgw_pfg_params;
#define PGW_PFG_MAX_REG 24     /* regulator terminal nodes (12 regulated phases) */

typedef struct pgw_pfg_tables {
  const pgw_pfg_elem* elem;  /* m                                                     */
  const double* W;           /* m x m complex (ld m): W_ik / (vb_i vb_k), W = -C Z C^T */
  const double* U0;          /* m complex, pu (EXACT: no-load; OPENDSS: direct solution) */
  const double* Gc;          /* OPENDSS check rows: n_chk x m complex (ld n_chk), pu     */
  const double* V0c;         /* n_chk complex, pu                                        */
  const double* G;           /* output rows: n_out x m complex (ld pad8(n_out)), pu      */
  const double* V0;          /* pad8(n_out) complex, pu                                  */
  const double* U_init;      /* optional EXACT initial guess, n x m complex env-major    */
  double* U_out;             /* optional final element voltages, n x m complex           */
  double* v_min_out;         /* optional min / max over the output rows (n)              */
  double* v_max_out;
  /* n_reg > 0 (RegControl): W / Gc / G carry n_reg extra columns (k = m ..
   * m + n_reg - 1: the rows' response to the correction currents c, pu per A) */
  const double* Greg;        /* x rows: n_reg x m complex (ld n_reg): G_R,k / (vb_k rho_j)  */
  const double* V0reg;       /* n_reg complex: V0_R / rho                                  */
  /* per env K(t), complex symmetric (D and S are), stored as its upper
   * triangle: K[i][l], i <= l, at [(i r_reg - i (i - 1) / 2 + l - i) n + e],
   * r_reg (r_reg + 1) / 2 complex */
  const double* Kreg;
  double* reg_x;             /* out: x per env, r_reg complex, [j n + e] (pu of rho)       */
  double* reg_c;             /* out: c per env, r_reg complex, [j n + e] (A)               */
  const int32_t* env_active; /* optional: envs with 0 are left untouched (control loop)   */
  const double* reg_rho;     /* r_reg (pgw_reg_params.rho): c = K (rho x)                */
} pgw_pfg_tables;

/* ctrl_p / ctrl_q: n_ctrl x n (NULL = 0); v_out: n_out x n (nullable); iters: n
 * (nullable; -count when stopped at max_iter unconverged). */
int32_t pgw_pf_solve_general(const pgw_pfg_params* p, const pgw_pfg_tables* t, int64_t n,
                             const double* ctrl_p, const double* ctrl_q, double* v_out,
                             int32_t* iters, void* stream);

/* ------------------------------------------------------------------------
 * RegControl (automatic regulator taps, OpenDSS RegControl in STATIC control
 * mode) on the general power flow.  A regulated phase is one phase of a
 * 2-winding transformer whose windings are wye to ground: its primitive
 * admittance over (a = winding-1 node, b = winding-2 node) is
 *   [[A / t1^2, B / (t1 t2)], [B / (t1 t2), C / t2^2]]
 * (A, B, C at unit taps; t1, t2 the winding taps, one of them the RegControl's
 * tap).  D(t) = Y(t) - Y(DSS taps) over R; K(t) = (I + D S)^-1 D with S =
 * U^T Z0 U, so that V(t) = V(DSS) - Z0 U K(t) U^T V(DSS) (Woodbury).
 * ---------------------------------------------------------------------- */
#define PGW_REG_MAX_PHASES 12
#define PGW_REG_MAX_CTRL 12
#define PGW_REG_MAX_MON 3
#define PGW_REG_PICK_PHASE 0
#define PGW_REG_PICK_MAX 1
#define PGW_REG_PICK_MIN 2
typedef struct pgw_reg_phase {
  int32_t a, b;              /* R indices of the winding-1 / winding-2 terminal     */
  int32_t ctrl;              /* the RegControl whose tap this phase follows          */
  int32_t tap_winding;       /* 1 or 2                                               */
  double A[2], B[2], C[2];   /* complex, siemens at unit taps                        */
  double tap1, tap2;         /* the DSS taps (those of Z0)                           */
} pgw_reg_phase;
typedef struct pgw_reg_ctrl {
  /* Sampled voltages: n_mon monitored phases, each an R node (the monitored
   * winding's terminal, or with Bus= the regulated bus's node) and the
   * pgw_reg_phase whose current is that phase's LDC current.  pick: which one
   * controls -- PGW_REG_PICK_PHASE the single entry (PTphase=k),
   * PGW_REG_PICK_MAX / _MIN the phase of largest / smallest |V| (PTphase=max /
   * min, the first on a tie). */
  int32_t n_mon, pick;
  int32_t mon_node[PGW_REG_MAX_MON];
  int32_t mon_phase[PGW_REG_MAX_MON];
  int32_t winding;           /* the monitored winding (1 or 2)                       */
  int32_t max_tap_change;    /* taps per control action                              */
  int32_t ldc;               /* 1: subtract (R + jX) I / ctprim (no Bus=)            */
  int32_t vlim_node;         /* Vlimit with Bus=: R index of the winding's first-phase
                                terminal; -1: the control voltage before LDC         */
  int32_t inverse_time;      /* 1: delay / min(10, 2 |vreg - v| / band)              */
  int32_t pad_;
  double vreg, band, ptratio, ctprim, r_ldc, x_ldc;  /* RegControl properties        */
  double vbase;              /* the winding's rated phase voltage / ptratio (V)      */
  double incr, min_tap, max_tap, delay;
  double vlimit;             /* Vlimit (V on the PT base; 0 = off)                   */
} pgw_reg_ctrl;
typedef struct pgw_reg_params {
  int32_t n_reg, r_reg;      /* as pgw_pfg_params                                    */
  int32_t n_phase, n_ctrl;
  pgw_reg_phase phase[PGW_REG_MAX_PHASES];
  pgw_reg_ctrl ctrl[PGW_REG_MAX_CTRL];
  const double* S;           /* r_reg x r_reg complex (ohm), row-major, device       */
  const double* rho;         /* r_reg: the volts per unit of x (node bases), device  */
} pgw_reg_params;

/* K(t) (packed as pgw_pfg_tables.Kreg) for the envs with active[e] != 0
 * (NULL: all), from the taps
 * (n_ctrl x n, the RegControls' present taps).  An env whose I + D S is
 * singular gets NaN in K, so its next solve reports unconverged. */
int32_t pgw_reg_factor(const pgw_reg_params* p, int64_t n, const double* taps, const int32_t* active,
                       double* Kreg, void* stream);
/* One control pass (RegControl.Sample + DoPendingAction, STATIC mode) after a
 * solve that wrote reg_x / reg_c: per env and RegControl, the monitored
 * voltage V / ptratio (PTphase=max / min: the phase of largest / smallest
 * |V|; Bus=: at the regulated bus), less the line-drop compensation
 * (R + jX) I / ctprim (not with Bus=), against vreg +- band / 2, and with
 * Vlimit the local voltage against vlimit (above it the boost is vlimit - V);
 * an acting control moves its tap by the needed change truncated to whole
 * steps (at least one, at most max_tap_change, inside [min_tap, max_tap]);
 * of the controls that act, only those with the smallest delay (inverse time:
 * delay / min(10, 2 |vreg - v| / band)) do so this pass.  active[e] = 1
 * where any tap moved (else 0); *n_changed (device int32) += that count. */
int32_t pgw_reg_control(const pgw_reg_params* p, int64_t n, const double* reg_x, const double* reg_c,
                        double* taps, int32_t* active, int32_t* n_changed, void* stream);

/* ------------------------------------------------------------------------
 * Kernel timing (benchmark instrumentation): while on, every `every`-th launch
 * of each kernel below is bracketed by HIP events on its own stream.
 * pgw_timing_stop synchronizes the recorded events and returns, per kernel,
 * the summed duration (ms) and the number of timed launches (PGW_T_COUNT
 * entries each).
 * ---------------------------------------------------------------------- */
enum { PGW_T_COORD_AGENTS = 0, PGW_T_COORD_PF = 1, PGW_T_PF_SOLVE = 2, PGW_T_RESERVED3 = 3,
       PGW_T_MA_STEP = 4, PGW_T_PF_GENERAL = 5, PGW_T_COUNT = 6 };
/* Debug: device buffer of 8 int64 per k_coord_pf / k_pf_solve wave (NULL = off); lane 0 of
 * each wave writes wall_clock64() (100 MHz) at its phase boundaries. */
int32_t pgw_debug_pf_trace(long long* buf);
/* Debug: device buffer of 128 int64 per block (16 waves x 8 slots) of k_mc_step /
 * k_ma_step (NULL = off); while set, pgw_mc_agent_step (fp64, unclocked) and
 * pgw_ma_step launch trace instantiations whose lane 0 of each wave writes
 * wall_clock64() (100 MHz) at its phase boundaries (pgw_components.hip). */
int32_t pgw_debug_mc_trace(long long* buf);
int32_t pgw_timing_start(int32_t every);
int32_t pgw_timing_stop(double* total_ms, int64_t* count);
/* Measured HBM ceiling (benchmark instrumentation): copies `bytes` (a multiple
 * of 16) from src to dst `reps` times with a 16-B-per-lane nontemporal copy
 * kernel and writes the average milliseconds per copy (2 x bytes of HBM
 * traffic).  Synchronizes. */
int32_t pgw_stream_copy(const void* src, void* dst, int64_t bytes, int32_t reps, float* ms_out,
                        void* stream);

/* ------------------------------------------------------------------------
 * Host-side feeder construction (C++, no GPU): the native stand-in for the
 * OpenDSS model build behind opendss.py:36-51.
 * ---------------------------------------------------------------------- */
/* PGW_ELEM_SHUNT: a constant admittance per phase, y_p = r[p] + j x[p] (siemens),
 * between node1[p] and node2[p] (-1 = ground): capacitors and constant-Z
 * (model 2) loads.
 * PGW_ELEM_XFMR_N: a 2- or 3-winding transformer with explicit terminals:
 * winding w of phase p spans wnode[(w * 3 + p) * 2] (hi) -> wnode[... + 1]
 * (lo, -1 = ground), so centre-tapped secondaries (bus.1.0 / bus.0.2) and
 * phase-to-phase single-phase windings are expressed directly.  The leakage
 * model is OpenDSS's N-winding one (Transformer.pas CalcY): short-circuit
 * impedances Z_ij = R_i + R_j + j X_ij on winding 1's kVA (R_k = %R_k / 100
 * referred from winding k's kVA), ZB = the (nw-1)^2 matrix of winding k+1
 * against winding 1, Y_pu = A ZB^-1 A^T (A: winding 1 row -1, the others the
 * identity), Y_ij = Y_pu,ij S_ph / (V_i V_j) with V_k = the winding's phase
 * voltage times its tap. */
enum { PGW_ELEM_LINE = 1, PGW_ELEM_XFMR = 2, PGW_ELEM_VSOURCE = 3, PGW_ELEM_SHUNT = 4, PGW_ELEM_XFMR_N = 5 };

typedef struct pgw_feeder_elem {
  int32_t kind;          /* PGW_ELEM_*                                     */
  int32_t nphases;
  int32_t node1[3];      /* terminal-1 node per phase (-1 = ground)        */
  int32_t node2[3];      /* terminal-2 node per phase (-1 = ground)        */
  int32_t conn1, conn2;  /* transformer winding connection: 0 wye, 1 delta */
  double r[9], x[9], c[9];  /* line: R, X (ohm/unit), C (nF/unit), row-major nphases^2 */
  double length;         /* line: length in the matrices' unit            */
  double freq;           /* Hz                                            */
  double kv1, kv2, kva, pct_r1, pct_r2, xhl;       /* transformer          */
  double tap1, tap2;     /* transformer winding taps (pu of kv, 0 = 1.0)  */
  double basekv, pu, angle, mvasc3, mvasc1, x1r1, x0r0;  /* vsource        */
  /* PGW_ELEM_XFMR_N (winding 1 and 2 use kv1 / kv2, pct_r1 / pct_r2, tap1 /
   * tap2, conn1 / conn2 and kva above; kva is winding 1's, the X base)    */
  int32_t nwindings;     /* 2 or 3                                         */
  int32_t conn3;
  int32_t wnode[18];     /* [winding][phase][hi, lo] terminal nodes        */
  double kv3, kva2, kva3, pct_r3, tap3, xht, xlt;  /* xht = X13, xlt = X23 (%) */
} pgw_feeder_elem;

/* Assemble the nodal admittance Y (n_nodes^2, complex interleaved, loads
 * excluded), Z = Y^-1, the source current injection and the no-load voltages
 * V0 = Z I_src.  Any output pointer may be NULL.  Host memory. */
int32_t pgw_feeder_build(const pgw_feeder_elem* elems, int32_t n_elems, int32_t n_nodes,
                         double* Y, double* Z, double* I_src, double* V0);
/* Reduce to the m load elements (element k spans node p[k] -> q[k], q = -1
 * ground): W = -C Z C^T, U0 = C V0, and for the n_out nodes in out_nodes:
 * G = -(Z C^T)[out_nodes], V0_out = V0[out_nodes].  Host memory. */
int32_t pgw_pf_reduce(int32_t n_nodes, const double* Z, const double* V0, int32_t m,
                      const int32_t* elem_p, const int32_t* elem_q, int32_t n_out,
                      const int32_t* out_nodes, double* W, double* U0, double* G,
                      double* V0_out);

/* ------------------------------------------------------------------------
 * Fused coordinated multi-building step (the BASELINE C4 hot path):
 * MultiAgentEnv.step (gridworld/multiagent_env.py:151-212) over n_agents
 * MultiComponentEnv agents of [building, pv, storage] (gridworld/scenarios/
 * buildings.py:11-72) + the power flow + CoordinatedMultiBuildingControlEnv.
 * reward_transform (examples/marl/openai/train.py:51-88), one thread per env.
 * ---------------------------------------------------------------------- */
#define PGW_MAX_AGENTS 8

typedef struct pgw_coord_params {
  pgw_building_params bld;
  pgw_pv_params pv;
  pgw_battery_params bat;
  double vv_lo, vv_hi, vv_penalty;   /* VOLTAGE_LIMITS, VV_UNIT_PENALTY         */
  int32_t n_agents;
  int32_t act_dim, obs_dim;          /* per agent                               */
  int32_t act_bld, act_pv, act_bat;  /* component action offsets (-1 = absent)  */
  int32_t obs_bld, obs_pv, obs_bat;  /* component obs offsets                   */
  int32_t comp_order[3];             /* 0 building, 1 pv, 2 storage             */
  int32_t n_comp;
  int32_t agent_ctrl[PGW_MAX_AGENTS];/* PF controllable slot of each agent's bus */
  int32_t coordinated;               /* apply the voltage-violation transform   */
  int32_t vv_row;                    /* PF output row of the common-bus voltage */
} pgw_coord_params;

/* Per-env buffers.  action: agent a's block at action.ptr + a * act_stride_agent;
 * obs likewise.  x: n_agents x 5 x n;  soc: n_agents x n;  reward, agent_power:
 * n_agents x n;  v_out: pf n_out x n;  vv: n (nullable). */
typedef struct pgw_coord_buffers {
  pgw_mat action; int64_t act_stride_agent;
  pgw_mat obs;    int64_t obs_stride_agent;
  double* x;
  double* soc;
  double* reward;
  double* agent_power;
  double* v_out;
  double* vv;
  int32_t* iters;
  /* OpenDSS rule with the hour's node records (pgw_pf_od.resp_v, output row 0
   * only): scratch for the envs the table does not serve -- od_list [n],
   * od_count [2] (zero-initialised once), od_parity flipped by the caller
   * every step (a step appends to od_count[parity] and zeroes the other).
   * Null: the two-kernel step (agents, then the PF kernel for every env). */
  int32_t* od_list;
  int32_t* od_count;
  int32_t od_parity, pad_;
} pgw_coord_buffers;

typedef struct pgw_coord_step_info {
  pgw_building_exo ex_t, ex_next;
  double pv_pmax;        /* PV data[index] before the advance */
} pgw_coord_step_info;

int32_t pgw_coord_step(const pgw_coord_params* p, const pgw_pf_params* pf,
                       const pgw_pf_tables* pft, const pgw_coord_step_info* s, int64_t n,
                       pgw_coord_buffers b, void* stream);

/* fp32-storage variant: every per-env buffer fp32, arithmetic in fp64 (the
 * power flow included: the agent powers are widened and summed in fp64, the
 * solve is the fp64 one).  Standard C4 agent layout only ([building, pv,
 * storage] at action offsets 0/6/7, default building obs) -- PGW_ERR_ARG
 * otherwise. */
typedef struct pgw_coord_buffers_f32 {
  pgw_matf action; int64_t act_stride_agent;
  pgw_matf obs;    int64_t obs_stride_agent;
  float* x;
  float* soc;
  float* reward;
  float* agent_power;
  float* v_out;
  float* vv;
  int32_t* iters;
} pgw_coord_buffers_f32;

/* The same coordinated step with the general power flow (pgw_pf_solve_general:
 * large feeders, OpenDSS's stopping rule): the agents' kernel, then the general
 * solve with the bus loads summed from agent_power (agent order) and the
 * coordinated voltage-violation epilogue on output row p->vv_row. */
int32_t pgw_coord_step_general(const pgw_coord_params* p, const pgw_pfg_params* pf,
                               const pgw_pfg_tables* pft, const pgw_coord_step_info* s, int64_t n,
                               pgw_coord_buffers b, void* stream);

int32_t pgw_coord_step_f32(const pgw_coord_params* p, const pgw_pf_params* pf,
                           const pgw_pf_tables* pft, const pgw_coord_step_info* s, int64_t n,
                           pgw_coord_buffers_f32 b, void* stream);

/* ------------------------------------------------------------------------
 * Fused MultiComponentEnv step (SURVEY 8(b) pgw_mc_agent_step): one agent of
 * building / PV / storage / EV components (each at most once, any order) --
 * MultiComponentEnv.step + step_reward (gridworld/base.py:114-156) with every
 * component's step (the entries above) and the in-order sums in ONE launch.
 * Same arithmetic as the separate kernels + pgw_agent_reduce (bit-identical).
 * The building's reward is the fresh one (MC semantics, base.py:137).
 * ---------------------------------------------------------------------- */
enum { PGW_MC_BUILDING = 0, PGW_MC_PV = 1, PGW_MC_STORAGE = 2, PGW_MC_EV = 3 };

typedef struct pgw_mc_component {
  int32_t kind, pad_;
  pgw_mat action;         /* the component's [N, act_dim] action            */
  pgw_mat obs;            /* its [N, obs_dim] observation                   */
  double* real_power;     /* its real power (building: p_consumed)          */
} pgw_mc_component;

/* One episode step's shared values for a device-clocked step (below): the
 * per-step fields of pgw_mc_step_args, one record per episode step in a device
 * table. */
typedef struct pgw_mc_step_dyn {
  pgw_building_exo bld_ex_t, bld_ex_next;
  pgw_ev_step_info ev_step;
  double pv_pmax, pad_;
} pgw_mc_step_dyn;

typedef struct pgw_mc_step_args {
  int32_t n_comp, pad_;
  pgw_mc_component comp[4];
  pgw_building_params bld;
  pgw_building_exo bld_ex_t, bld_ex_next;
  pgw_building_ext bld_ext;
  double* bld_x;
  double* bld_reward_state;
  pgw_pv_params pv;
  double pv_pmax;
  const double* pv_min_voltage;
  pgw_battery_params bat;
  double* bat_soc;
  pgw_ev_params ev;
  pgw_ev_step_info ev_step;
  const double* ev_endp;
  double* ev_req;
  uint64_t* ev_charging;
  double* ev_reward;
  double* real_power;     /* agent sums (n)                                 */
  double* reward;
  /* Device clock (optional, NULL = none; makes the launch's arguments the same
   * at every step, so a captured hipGraph of it can be replayed step after
   * step): one int32 per block of 64 envs, clock[b] = the episode step k of
   * block b, read at launch and advanced by one by that block.  The step's
   * shared values then come from dyn[min(k, n_dyn - 1)] (n_dyn records, built
   * by the caller with the values it would pass per step) instead of
   * bld_ex_t / bld_ex_next / pv_pmax / ev_step.  clock and dyn are both given
   * or both NULL. */
  const pgw_mc_step_dyn* dyn;
  int32_t* clock;
  int32_t n_dyn, pad2_;
} pgw_mc_step_args;

int32_t pgw_mc_agent_step(const pgw_mc_step_args* a, int64_t n, void* stream);

/* fp32 storage variant: the same fields, every per-env buffer
 * (state, obs, actions, real powers, rewards) fp32; fp64 arithmetic, each value
 * rounded once at its store, the agent sums formed in fp64 from the
 * components' stored values (what pgw_agent_reduce would read).  ev_endp,
 * ev_charging and pv_min_voltage keep their types.  Layout-identical to
 * pgw_mc_step_args. */
typedef struct pgw_mc_component_f32 {
  int32_t kind, pad_;
  pgw_matf action;
  pgw_matf obs;
  float* real_power;
} pgw_mc_component_f32;

typedef struct pgw_mc_step_args_f32 {
  int32_t n_comp, pad_;
  pgw_mc_component_f32 comp[4];
  pgw_building_params bld;
  pgw_building_exo bld_ex_t, bld_ex_next;
  pgw_building_ext bld_ext;
  float* bld_x;
  float* bld_reward_state;
  pgw_pv_params pv;
  double pv_pmax;
  const double* pv_min_voltage;
  pgw_battery_params bat;
  float* bat_soc;
  pgw_ev_params ev;
  pgw_ev_step_info ev_step;
  const double* ev_endp;
  float* ev_req;
  uint64_t* ev_charging;
  float* ev_reward;
  float* real_power;
  float* reward;
  const pgw_mc_step_dyn* dyn;
  int32_t* clock;
  int32_t n_dyn, pad2_;
} pgw_mc_step_args_f32;

int32_t pgw_mc_agent_step_f32(const pgw_mc_step_args_f32* a, int64_t n, void* stream);

/* Test / A-B knob of pgw_mc_agent_step's EV walk (process-wide, not per call):
 * -1 = automatic (the default: split over extra waves where the blocks are at
 * most one per CU and the step's scan has 2+ chunks), 0 = always in one lane,
 * 1 = always split.  Results are bit-identical in every mode.  The library
 * reads PGW_MC_EV_SPLIT=0/1 once, at load, as the initial mode.  *previous
 * (nullable) receives the mode it replaces. */
int32_t pgw_mc_ev_split_mode(int32_t mode, int32_t* previous);

/* ------------------------------------------------------------------------
 * Captured launches (hipGraph; the reference has no equivalent -- its step is
 * a Python call chain): every launch the library issues on `stream` between
 * pgw_graph_begin and pgw_graph_end becomes one executable graph (*exec_out),
 * replayed with pgw_graph_launch on any stream.  A launch's arguments are
 * frozen at capture: capture steps whose arguments do not change per step
 * (pgw_mc_step_args with clock / dyn, pgw_battery_step).  The stream must be a
 * created stream (not the null stream); capture mode is thread-local.
 * ---------------------------------------------------------------------- */
int32_t pgw_graph_begin(void* stream);
int32_t pgw_graph_end(void* stream, void** exec_out);
int32_t pgw_graph_launch(void* exec, void* stream);
int32_t pgw_graph_destroy(void* exec);

/* ------------------------------------------------------------------------
 * Fused multi-agent step over MC-kind components (the heterogeneous scenario,
 * gridworld/scenarios/heterogeneous.py:13-112): MultiAgentEnv.step
 * (gridworld/multiagent_env.py:151-212) for agents that are plain
 * MultiComponentEnvs of the PGW_MC_* kinds or single PV / storage / EV envs,
 * the per-bus load sums (:171-181) and the power flow -- two launches, one call.
 * The component slots (at most PGW_MA_MAX_SLOTS over all agents, agents'
 * slots contiguous and in component order) share ONE parameter set per kind,
 * as in pgw_mc_step_args, except PV which has two (pv, pv2): at most one
 * building, one storage and one EV component in total.
 * A block of 64 envs runs n_waves waves, wave w stepping the slots
 * wave_slot[wave_first[w] .. + wave_count[w]) one after another (e.g. one wave
 * per building / EV slot, the light PV / storage slots together); after the
 * block barrier wave 0 forms every agent's sums (0 + c0 + c1 ..., component
 * order, base.py:125-156) and every bus's load (0 + a0 + a1 ..., agent order).
 * ---------------------------------------------------------------------- */
#define PGW_MA_MAX_SLOTS 8

typedef struct pgw_ma_step_args {
  int32_t n_comp, pad_;                     /* component slots                        */
  pgw_mc_component comp[PGW_MA_MAX_SLOTS];  /* kind, action, obs, real_power per slot */
  /* parameter sets, state and per-step values: the pgw_mc_step_args fields */
  pgw_building_params bld;
  pgw_building_exo bld_ex_t, bld_ex_next;
  pgw_building_ext bld_ext;
  double* bld_x;
  double* bld_reward_state;
  pgw_pv_params pv;
  double pv_pmax;
  const double* pv_min_voltage;
  pgw_battery_params bat;
  double* bat_soc;
  pgw_ev_params ev;
  pgw_ev_step_info ev_step;
  const double* ev_endp;
  double* ev_req;
  uint64_t* ev_charging;
  double* ev_reward;
  /* second PV parameter set (slot_pv2[c] = 1) */
  pgw_pv_params pv2;
  double pv2_pmax;
  const double* pv2_min_voltage;
  /* per slot: owning agent; PV parameter set; PV band reward output (NULL =
   * none): -(band_scale (min(0, v - band_lo) + min(0, band_hi - v)))^2 of the
   * PV's min_voltage v (ThisPVEnv.step_reward, heterogeneous.py:47-52) */
  int32_t slot_agent[PGW_MA_MAX_SLOTS];
  int32_t slot_pv2[PGW_MA_MAX_SLOTS];
  double* slot_reward[PGW_MA_MAX_SLOTS];
  double band_lo, band_hi, band_scale;
  /* agents: slots [first, first + count); bus = controllable-load slot of its
   * bus (-1: none); sum = 1 for a MultiComponentEnv (real_power / reward get
   * the in-order sums), 0 for a single component (its own buffers are the
   * agent's) */
  int32_t n_agents, n_bus;
  int32_t agent_first[PGW_MAX_AGENTS], agent_count[PGW_MAX_AGENTS];
  int32_t agent_bus[PGW_MAX_AGENTS], agent_sum[PGW_MAX_AGENTS];
  double* agent_real_power[PGW_MAX_AGENTS];
  double* agent_reward[PGW_MAX_AGENTS];
  double* bus_p;                            /* n_bus x n bus loads (kW)               */
  /* waves of a block: each slot listed once in wave_slot */
  int32_t n_waves, pad2_;
  int32_t wave_first[PGW_MA_MAX_SLOTS], wave_count[PGW_MA_MAX_SLOTS];
  int32_t wave_slot[PGW_MA_MAX_SLOTS];
} pgw_ma_step_args;

/* The agents' step (k_ma_step), then -- pf != NULL -- pgw_pf_solve(pf, pft, n,
 * a->bus_p, NULL, v_out, iters) on the same stream (pf->n_ctrl == a->n_bus).
 * v_out may be NULL when pft carries v_min_out / v_max_out (extrema only). */
int32_t pgw_ma_step(const pgw_ma_step_args* a, const pgw_pf_params* pf, const pgw_pf_tables* pft,
                    int64_t n, double* v_out, int32_t* iters, void* stream);

/* ------------------------------------------------------------------------
 * Home-Steward house: HSMultiComponentEnv.reset/step
 * (gridworld/base_hs.py:66-180) over its components HSPVEnv
 * (pv_profile_env_hs.py:96-160), HSEnergyStorageEnv
 * (energy_storage_env_hs.py:76-270), HSEVChargingEnv
 * (ev_charging_env_hs.py:127-326) and HSDevicesEnv (devices_env_hs.py:106-205).
 * One thread per env runs the components in chain order and passes the step's
 * resource state (PV / battery / grid power still available) down the chain
 * as the reference's meta_state does; the house reward is then evaluated from
 * the final state (base_hs.py:163, 183-199).
 * ---------------------------------------------------------------------- */
#define PGW_HS_MAX_VEHICLES 64
#define PGW_HS_MAX_DEV 4
enum { PGW_HS_PV = 0, PGW_HS_STORAGE = 1, PGW_HS_EV = 2, PGW_HS_DEVICES = 3 };

typedef struct pgw_hs_params {
  int32_t n_comp;                 /* components in chain order, each kind at most once */
  int32_t kind[4];                /* PGW_HS_*                                 */
  int32_t obs_off[4];             /* obs column of each chain slot's block    */
  int32_t rescale[4];             /* rescale_spaces of each chain slot        */
  int32_t n_veh, n_dev;
  /* PV: action box (0.98, 1), obs box (-max(data), 0) */
  double pv_act_low, pv_act_high, pv_obs_low;
  /* storage */
  double soc_min, soc_max, eta_c, eta_d, max_power, dt_h, max_storage_cost;
  /* EV */
  double ev_rate, ev_hours_per_step, ev_steps_per_hour, ev_mult, ev_unserved_penalty;
  double ev_obs_low[7], ev_obs_high[7];
  double ev_end_park[PGW_HS_MAX_VEHICLES];    /* rounded end_time_park_min */
  double ev_req0[PGW_HS_MAX_VEHICLES];        /* energy_required_kwh * multiplier */
  /* devices: action box (0.99, 1), obs box (0, column max) */
  double dev_act_low, dev_act_high, dev_hours_per_step;
  double dev_obs_high[PGW_HS_MAX_DEV];
  double max_grid_power;
  uint64_t* oob;                  /* nullable device counter, see PGW_OOB     */
  int32_t pv_grid_aware;          /* HSPVEnv(grid_aware): obs + min_voltage (0.9, 1.1) */
  int32_t pad_;
} pgw_hs_params;

/* Per-step values shared by all envs (the house steps in lockstep). */
typedef struct pgw_hs_step_info {
  double pv_avail;                 /* PV data[index] (scaled)                  */
  double grid_cost;                /* grid_cost[time_index]                    */
  double dev_obs[PGW_HS_MAX_DEV];  /* devices data row (scaled), obs          */
  double dev_power[PGW_HS_MAX_DEV];/* devices data_pd row, summed for power   */
  double ev_time;                  /* EV loop time (minutes)                   */
  double ev_next_time;             /* simulation_times[time_index]             */
  uint64_t ev_window;              /* bit v: start_v <= ev_time <= end_park_v  */
} pgw_hs_step_info;

/* Per-device step_meta records (base_hs.py:133-164 collects one dict per
 * chain slot: pv_profile_env_hs.py:151-170, energy_storage_env_hs.py:180-185,
 * 257-265, ev_charging_env_hs.py:172-180, 316-320, devices_env_hs.py:129-137,
 * 195-199).  Numeric fields, each an n-vector at
 * step_meta[(slot * PGW_HS_META_FIELDS + field) * n + e]:
 *   0 cost, 1 reward (the component's own, with the meta_state of its step),
 *   2 action (raw, after to_raw), 3 solar_power_consumed,
 *   4 es_power_consumed, 5 grid_power_consumed,
 *   6.. device_custom_info in the reference's key order:
 *     PV       pv_available_power, pv_actionable_power
 *     storage  current_storage, power_ask, solar_power_available,
 *              grid_power_available, es_power_available
 *     EV       power_ask, power_unserved, charging_vehicle, vehicle_charged,
 *              solar_power_available, es_power_available, grid_power_available
 *     devices  power_ask, solar_power_available, es_power_available,
 *              grid_power_available
 * (device_id and timestamp are host strings).  Unused fields are not written. */
#define PGW_HS_META_FIELDS 13

/* Per-env state and outputs (device).  action: n x n_comp, column = chain
 * slot.  obs: n x obs_dim.  ev_req: n_veh x n.  es_power_last: the house's
 * meta_state es_power, which survives into the next reset's EV step.
 * meta_out (nullable): 3 x n final pv_power, es_power, grid_power.
 * step_meta (nullable, step only): n_comp x PGW_HS_META_FIELDS x n records. */
typedef struct pgw_hs_buffers {
  pgw_mat action;
  pgw_mat obs;
  double* soc;
  double* soc_cost;        /* storage current_cost (not reset by reset)   */
  double* ev_req;
  uint64_t* ev_charging;   /* bit v: vehicle v charged at the last step   */
  double* ev_cost;         /* EV current_cost                             */
  double* dev_cost;        /* devices current_cost                        */
  double* es_power_last;
  double* reward;
  double* real_power;
  double* meta_out;
  double* step_meta;
  /* meta_state pv_power carried from step to step (base_hs.py keeps one
   * meta_state dict: a component ahead of the PV in the chain sees the last
   * step's final pv_power; NaN stands for the reference's initial None).
   * NULL: 0 at every step start (a PV-first chain never reads it). */
  double* pv_power_last;
  const double* min_voltage;  /* n, the grid-aware PV's observation (NULL otherwise) */
} pgw_hs_buffers;

/* reset (base_hs.py:66-91): PV and devices at row 0, storage SoC := clip(
 * init_soc[e]) (n doubles, device), EV requirements restored and its
 * action-less step, obs of every component.  s: the reset row's values. */
int32_t pgw_hs_reset(const pgw_hs_params* p, const pgw_hs_step_info* s, int64_t n,
                     const double* init_soc, pgw_hs_buffers b, void* stream);
/* step (base_hs.py:114-180): the chain, obs, real_power (sum in chain order)
 * and the house reward. */
int32_t pgw_hs_step(const pgw_hs_params* p, const pgw_hs_step_info* s, int64_t n,
                    pgw_hs_buffers b, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* PGW_H_ */
