"""ctypes binding of libpgw.so (the C ABI declared in include/pgw.h).

There is no fallback: if the in-tree library is missing or stale the import
fails loudly -- the product path never silently runs anything but the HIP
kernels.
"""
import ctypes as C
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# PGW_LIB_PATH: another build of the same ABI (same-box A/B measurements only)
LIB_PATH = os.environ.get("PGW_LIB_PATH") or os.path.join(_HERE, "libpgw.so")
ABI_VERSION = 31

f64, i32, i64, u64, vp = C.c_double, C.c_int32, C.c_int64, C.c_uint64, C.c_void_p
P = C.POINTER

BLD_MAX_OBS = 24
EV_MAX_WORDS = 16
MAX_COMP = 8
PF_MAX_M = 16
PF_MAX_CTRL = 8
PFG_MAX_M = 128
PFG_MAX_CHK = 256
MAX_AGENTS = 8


class PgwError(RuntimeError):
    pass


class Mat(C.Structure):
    _fields_ = [("ptr", vp), ("s_env", i64), ("s_dim", i64)]


class Matf(C.Structure):
    """pgw_matf: the fp32-storage variant of Mat (the *_f32 entries)."""
    _fields_ = [("ptr", vp), ("s_env", i64), ("s_dim", i64)]


class BatteryParams(C.Structure):
    _fields_ = [("soc_min", f64), ("soc_max", f64), ("eta_c", f64), ("eta_d", f64),
                ("max_power", f64), ("dt_h", f64), ("rescale", i32), ("sampled_init", i32),
                ("oob", vp)]


class PVParams(C.Structure):
    _fields_ = [("obs_low", f64), ("obs_high", f64), ("vmin_low", f64), ("vmin_high", f64),
                ("rescale", i32), ("grid_aware", i32), ("oob", vp)]


class BuildingParams(C.Structure):
    _fields_ = [("A", f64 * 5), ("B", (f64 * 4) * 5), ("K", f64 * 5), ("C", f64 * 5),
                ("mean", f64 * 5), ("act_low", f64 * 6), ("act_high", f64 * 6),
                ("T_init", f64 * 5), ("obs_low", f64 * BLD_MAX_OBS),
                ("obs_high", f64 * BLD_MAX_OBS), ("alpha", f64),
                ("sel", (i32 * 4) * 5), ("nbr", (i32 * 4) * 5),
                ("obs_var", i32 * BLD_MAX_OBS), ("n_obs", i32), ("rescale", i32),
                ("oob", vp)]


class BuildingExo(C.Structure):
    _fields_ = [("T_oa", f64), ("q_solar", f64 * 5), ("q_int", f64 * 5), ("q_cool", f64 * 5),
                ("comfort_lb", f64), ("comfort_ub", f64), ("time_of_day", f64), ("pad_", f64)]


class BuildingExt(C.Structure):
    _fields_ = [("bus_voltage", vp), ("min_voltage", vp), ("max_voltage", vp), ("p_setpoint", vp)]


class EVParams(C.Structure):
    _fields_ = [("rate", f64), ("hours_per_step", f64), ("mult", f64), ("u_pen", f64),
                ("p_pen", f64), ("thr", f64), ("reward_scale", f64), ("obs_low", f64 * 6),
                ("obs_high", f64 * 6), ("n_vehicles", i32), ("rescale", i32), ("oob", vp)]


class EVStepInfo(C.Structure):
    _fields_ = [("time", f64), ("next_time", f64), ("action_default", f64), ("tl_rcp", vp),
                ("env_start", vp), ("env_endp", vp), ("n_words", i32),
                ("pad_", i32), ("window", u64 * EV_MAX_WORDS), ("scan", u64 * EV_MAX_WORDS)]


class ReduceArgs(C.Structure):
    _fields_ = [("real_power", vp * MAX_COMP), ("reward", vp * MAX_COMP), ("n_comp", i32),
                ("pad_", i32)]


class PFParams(C.Structure):
    _fields_ = [("vbase", f64 * PF_MAX_M), ("vmin", f64 * PF_MAX_M), ("vmax", f64 * PF_MAX_M),
                ("vlow", f64 * PF_MAX_M), ("nph", f64 * PF_MAX_M), ("base_kw", f64 * PF_MAX_M),
                ("base_kvar", f64 * PF_MAX_M), ("tol", f64), ("pred_x0", f64), ("pred_h", f64),
                ("elem_ctrl", i32 * PF_MAX_M),
                ("m", i32), ("n_ctrl", i32), ("n_out", i32), ("max_iter", i32), ("pred_n", i32),
                ("pad_", i32)]


class PFTables(C.Structure):
    _fields_ = [("block", vp), ("G", vp), ("V0", vp), ("U_pred", vp),
                ("U_pred_meta", vp), ("U_init", vp), ("U_out", vp), ("sig_out", vp),
                ("load_scale", vp), ("v_min_out", vp), ("v_max_out", vp), ("od", vp)]


PF_OD_MAX_ROWS = 28


class PFOD(C.Structure):
    _fields_ = [("tol", f64), ("y0r", f64 * PF_MAX_M), ("y0i", f64 * PF_MAX_M),
                ("elem_scale", f64 * PF_MAX_M), ("gamma", f64), ("eps", f64), ("gmax", f64),
                ("gsrc", f64), ("min_iter", i32), ("n_rep", i32), ("n_rows", i32), ("sparse_envs", i32),
                ("rows_V0", vp), ("rows_G", vp), ("start", vp), ("resp", vp), ("resp_x0", f64),
                ("resp_h", f64), ("resp_nseg", i32), ("resp_v_row", i32), ("resp_v", vp), ("resp_rows", u64),
                ("resp_q", vp), ("resp_q_rows", u64), ("resp_q_stride", i32), ("resp_q_k", i32)]


OD_REC_HEAD = 6
OD_VREC = 12                     # doubles per node record (PGW_OD_VREC)


def od_rec(m):
    """Doubles per response-table record (PGW_OD_REC)."""
    return OD_REC_HEAD + 6 * m


class PFGElem(C.Structure):
    _fields_ = [("base_kw", f64), ("base_kvar", f64), ("nph", f64), ("y0r", f64), ("y0i", f64),
                ("vlo2", f64), ("vmn2", f64), ("vmx2", f64), ("ctrl", i32), ("model", i32),
                ("exp_p", f64), ("exp_q", f64), ("zip", f64 * 6), ("vcut2", f64)]


class PFGParams(C.Structure):
    _fields_ = [("m", i32), ("n_chk", i32), ("n_out", i32), ("n_ctrl", i32), ("mode", i32),
                ("min_iter", i32), ("max_iter", i32), ("pad_", i32), ("tol", f64), ("coef", f64),
                ("rescale", f64), ("n_reg", i32), ("r_reg", i32)]


class PFGTables(C.Structure):
    _fields_ = [("elem", vp), ("W", vp), ("U0", vp), ("Gc", vp), ("V0c", vp), ("G", vp), ("V0", vp),
                ("U_init", vp), ("U_out", vp), ("v_min_out", vp), ("v_max_out", vp),
                ("Greg", vp), ("V0reg", vp), ("Kreg", vp), ("reg_x", vp), ("reg_c", vp),
                ("env_active", vp), ("reg_rho", vp)]


PFG_MAX_REG, REG_MAX_PHASES, REG_MAX_CTRL, REG_MAX_MON = 24, 12, 12, 3
REG_PICK_PHASE, REG_PICK_MAX, REG_PICK_MIN = 0, 1, 2


class RegPhase(C.Structure):
    _fields_ = [("a", i32), ("b", i32), ("ctrl", i32), ("tap_winding", i32), ("A", f64 * 2),
                ("B", f64 * 2), ("C", f64 * 2), ("tap1", f64), ("tap2", f64)]


class RegCtrl(C.Structure):
    _fields_ = [("n_mon", i32), ("pick", i32), ("mon_node", i32 * REG_MAX_MON),
                ("mon_phase", i32 * REG_MAX_MON), ("winding", i32), ("max_tap_change", i32), ("ldc", i32),
                ("vlim_node", i32), ("inverse_time", i32), ("pad_", i32),
                ("vreg", f64), ("band", f64), ("ptratio", f64), ("ctprim", f64), ("r_ldc", f64),
                ("x_ldc", f64), ("vbase", f64), ("incr", f64), ("min_tap", f64), ("max_tap", f64),
                ("delay", f64), ("vlimit", f64)]


class RegParams(C.Structure):
    _fields_ = [("n_reg", i32), ("r_reg", i32), ("n_phase", i32), ("n_ctrl", i32),
                ("phase", RegPhase * REG_MAX_PHASES), ("ctrl", RegCtrl * REG_MAX_CTRL), ("S", vp),
                ("rho", vp)]


PF_EXACT, PF_OPENDSS, PF_OPENDSS_STEP = 0, 1, 2


class PredMeta(C.Structure):
    _fields_ = [("tstar", f64), ("left", i32), ("right", i32)]


class FeederElem(C.Structure):
    _fields_ = [("kind", i32), ("nphases", i32), ("node1", i32 * 3), ("node2", i32 * 3),
                ("conn1", i32), ("conn2", i32), ("r", f64 * 9), ("x", f64 * 9), ("c", f64 * 9),
                ("length", f64), ("freq", f64), ("kv1", f64), ("kv2", f64), ("kva", f64),
                ("pct_r1", f64), ("pct_r2", f64), ("xhl", f64), ("tap1", f64), ("tap2", f64),
                ("basekv", f64), ("pu", f64),
                ("angle", f64), ("mvasc3", f64), ("mvasc1", f64), ("x1r1", f64), ("x0r0", f64),
                ("nwindings", i32), ("conn3", i32), ("wnode", i32 * 18), ("kv3", f64), ("kva2", f64),
                ("kva3", f64), ("pct_r3", f64), ("tap3", f64), ("xht", f64), ("xlt", f64)]


class CoordParams(C.Structure):
    _fields_ = [("bld", BuildingParams), ("pv", PVParams), ("bat", BatteryParams),
                ("vv_lo", f64), ("vv_hi", f64), ("vv_penalty", f64), ("n_agents", i32),
                ("act_dim", i32), ("obs_dim", i32), ("act_bld", i32), ("act_pv", i32),
                ("act_bat", i32), ("obs_bld", i32), ("obs_pv", i32), ("obs_bat", i32),
                ("comp_order", i32 * 3), ("n_comp", i32), ("agent_ctrl", i32 * MAX_AGENTS),
                ("coordinated", i32), ("vv_row", i32)]


class CoordBuffers(C.Structure):
    _fields_ = [("action", Mat), ("act_stride_agent", i64), ("obs", Mat), ("obs_stride_agent", i64),
                ("x", vp), ("soc", vp), ("reward", vp), ("agent_power", vp), ("v_out", vp),
                ("vv", vp), ("iters", vp), ("od_list", vp), ("od_count", vp), ("od_parity", i32),
                ("pad_", i32)]


class CoordBuffersF32(C.Structure):
    _fields_ = [("action", Matf), ("act_stride_agent", i64), ("obs", Matf), ("obs_stride_agent", i64),
                ("x", vp), ("soc", vp), ("reward", vp), ("agent_power", vp), ("v_out", vp),
                ("vv", vp), ("iters", vp)]


class CoordStepInfo(C.Structure):
    _fields_ = [("ex_t", BuildingExo), ("ex_next", BuildingExo), ("pv_pmax", f64)]


HS_MAX_VEHICLES, HS_MAX_DEV = 64, 4


class MCComponent(C.Structure):
    _fields_ = [("kind", i32), ("pad_", i32), ("action", Mat), ("obs", Mat), ("real_power", vp)]


class MCStepDyn(C.Structure):
    """pgw_mc_step_dyn: one episode step's shared values (device table record)."""
    _fields_ = [("bld_ex_t", BuildingExo), ("bld_ex_next", BuildingExo), ("ev_step", EVStepInfo),
                ("pv_pmax", f64), ("pad_", f64)]


class MCStepArgs(C.Structure):
    _fields_ = [("n_comp", i32), ("pad_", i32), ("comp", MCComponent * 4),
                ("bld", BuildingParams), ("bld_ex_t", BuildingExo), ("bld_ex_next", BuildingExo),
                ("bld_ext", BuildingExt), ("bld_x", vp), ("bld_reward_state", vp),
                ("pv", PVParams), ("pv_pmax", f64), ("pv_min_voltage", vp),
                ("bat", BatteryParams), ("bat_soc", vp),
                ("ev", EVParams), ("ev_step", EVStepInfo), ("ev_endp", vp), ("ev_req", vp),
                ("ev_charging", vp), ("ev_reward", vp), ("real_power", vp), ("reward", vp),
                ("dyn", vp), ("clock", vp), ("n_dyn", i32), ("pad2_", i32)]


class MCComponentF32(C.Structure):
    _fields_ = [("kind", i32), ("pad_", i32), ("action", Matf), ("obs", Matf), ("real_power", vp)]


class MCStepArgsF32(C.Structure):
    """pgw_mc_step_args_f32: pgw_mc_step_args with fp32 per-env buffers (the same
    field names, so the components' _mc_static / _mc_prepare fill it unchanged)."""
    _fields_ = [(nm, MCComponentF32 * 4) if nm == "comp" else (nm, tp) for nm, tp in MCStepArgs._fields_]


MA_MAX_SLOTS = 8


class MAStepArgs(C.Structure):
    """pgw_ma_step_args: the pgw_mc_step_args fields (same names, so the
    components' _mc_static / _mc_prepare fill it unchanged) with 8 slots, a
    second PV parameter set and the agent / bus layout."""
    _fields_ = [("n_comp", i32), ("pad_", i32), ("comp", MCComponent * MA_MAX_SLOTS),
                ("bld", BuildingParams), ("bld_ex_t", BuildingExo), ("bld_ex_next", BuildingExo),
                ("bld_ext", BuildingExt), ("bld_x", vp), ("bld_reward_state", vp),
                ("pv", PVParams), ("pv_pmax", f64), ("pv_min_voltage", vp),
                ("bat", BatteryParams), ("bat_soc", vp),
                ("ev", EVParams), ("ev_step", EVStepInfo), ("ev_endp", vp), ("ev_req", vp),
                ("ev_charging", vp), ("ev_reward", vp),
                ("pv2", PVParams), ("pv2_pmax", f64), ("pv2_min_voltage", vp),
                ("slot_agent", i32 * MA_MAX_SLOTS), ("slot_pv2", i32 * MA_MAX_SLOTS),
                ("slot_reward", vp * MA_MAX_SLOTS), ("band_lo", f64), ("band_hi", f64), ("band_scale", f64),
                ("n_agents", i32), ("n_bus", i32),
                ("agent_first", i32 * MAX_AGENTS), ("agent_count", i32 * MAX_AGENTS),
                ("agent_bus", i32 * MAX_AGENTS), ("agent_sum", i32 * MAX_AGENTS),
                ("agent_real_power", vp * MAX_AGENTS), ("agent_reward", vp * MAX_AGENTS), ("bus_p", vp),
                ("n_waves", i32), ("pad2_", i32), ("wave_first", i32 * MA_MAX_SLOTS),
                ("wave_count", i32 * MA_MAX_SLOTS), ("wave_slot", i32 * MA_MAX_SLOTS)]


class HSParams(C.Structure):
    _fields_ = [("n_comp", i32), ("kind", i32 * 4), ("obs_off", i32 * 4), ("rescale", i32 * 4),
                ("n_veh", i32), ("n_dev", i32),
                ("pv_act_low", f64), ("pv_act_high", f64), ("pv_obs_low", f64),
                ("soc_min", f64), ("soc_max", f64), ("eta_c", f64), ("eta_d", f64), ("max_power", f64),
                ("dt_h", f64), ("max_storage_cost", f64),
                ("ev_rate", f64), ("ev_hours_per_step", f64), ("ev_steps_per_hour", f64), ("ev_mult", f64),
                ("ev_unserved_penalty", f64), ("ev_obs_low", f64 * 7), ("ev_obs_high", f64 * 7),
                ("ev_end_park", f64 * HS_MAX_VEHICLES), ("ev_req0", f64 * HS_MAX_VEHICLES),
                ("dev_act_low", f64), ("dev_act_high", f64), ("dev_hours_per_step", f64),
                ("dev_obs_high", f64 * HS_MAX_DEV), ("max_grid_power", f64), ("oob", vp),
                ("pv_grid_aware", i32), ("pad_", i32)]


class HSStepInfo(C.Structure):
    _fields_ = [("pv_avail", f64), ("grid_cost", f64), ("dev_obs", f64 * HS_MAX_DEV),
                ("dev_power", f64 * HS_MAX_DEV), ("ev_time", f64), ("ev_next_time", f64),
                ("ev_window", C.c_uint64)]


class HSBuffers(C.Structure):
    _fields_ = [("action", Mat), ("obs", Mat), ("soc", vp), ("soc_cost", vp), ("ev_req", vp),
                ("ev_charging", vp), ("ev_cost", vp), ("dev_cost", vp), ("es_power_last", vp),
                ("reward", vp), ("real_power", vp), ("meta_out", vp), ("step_meta", vp),
                ("pv_power_last", vp), ("min_voltage", vp)]


PGW_ELEM_LINE, PGW_ELEM_XFMR, PGW_ELEM_VSOURCE, PGW_ELEM_SHUNT, PGW_ELEM_XFMR_N = 1, 2, 3, 4, 5

_SIGS = {
    "pgw_abi_version": (i32, []),
    "pgw_struct_sizes": (i32, [P(i64), i32]),
    "pgw_pf_od_probe_args_size": (i64, [i32]),
    "pgw_pf_od_probe": (i32, [P(PFParams), i32, P(PFTables), vp, i32, i64, vp, vp, vp, vp, vp, vp]),
    "pgw_pf_od_resp_fit": (i32, [i32, i64, vp, vp, vp, vp, vp, vp, vp]),
    "pgw_pf_od_resp_check": (i32, [i32, i64, vp, vp, vp, vp, vp, vp, vp]),
    "pgw_last_error": (C.c_char_p, []),
    "pgw_battery_reset": (i32, [P(BatteryParams), i64, vp, vp, Mat, vp]),
    "pgw_battery_step": (i32, [P(BatteryParams), i64, Mat, vp, Mat, vp, vp]),
    "pgw_battery_reset_f32": (i32, [P(BatteryParams), i64, vp, vp, Matf, vp]),
    "pgw_battery_step_f32": (i32, [P(BatteryParams), i64, Matf, vp, Matf, vp, vp]),
    "pgw_pv_obs": (i32, [P(PVParams), i64, f64, vp, Mat, vp]),
    "pgw_pv_step": (i32, [P(PVParams), i64, f64, Mat, vp, Mat, vp, vp]),
    "pgw_building_reset": (i32, [P(BuildingParams), P(BuildingExo), i64, vp, vp, vp, BuildingExt,
                                 Mat, vp]),
    "pgw_building_step": (i32, [P(BuildingParams), P(BuildingExo), P(BuildingExo), i64, Mat, vp, vp,
                                vp, vp, i32, BuildingExt, Mat, vp]),
    "pgw_ev_reset": (i32, [P(EVParams), i64, vp, vp, vp, vp]),
    "pgw_ev_reset_tables": (i32, [P(EVParams), i64, vp, vp, vp, vp]),
    "pgw_pv_obs_f32": (i32, [P(PVParams), i64, f64, vp, Matf, vp]),
    "pgw_pv_step_f32": (i32, [P(PVParams), i64, f64, Matf, vp, Matf, vp, vp]),
    "pgw_building_reset_f32": (i32, [P(BuildingParams), P(BuildingExo), i64, vp, vp, vp, BuildingExt, Matf, vp]),
    "pgw_building_step_f32": (i32, [P(BuildingParams), P(BuildingExo), P(BuildingExo), i64, Matf, vp, vp, vp, vp,
                                    i32, BuildingExt, Matf, vp]),
    "pgw_ev_reset_f32": (i32, [P(EVParams), i64, vp, vp, vp, vp]),
    "pgw_ev_reset_tables_f32": (i32, [P(EVParams), i64, vp, vp, vp, vp]),
    "pgw_ev_step_f32": (i32, [P(EVParams), P(EVStepInfo), i64, Matf, vp, vp, vp, Matf, vp, vp, vp]),
    "pgw_ev_step": (i32, [P(EVParams), P(EVStepInfo), i64, Mat, vp, vp, vp, Mat, vp, vp, vp]),
    "pgw_ev_step_lanes": (i32, [P(EVParams), P(EVStepInfo), i64, Mat, vp, vp, vp, Mat, vp, vp, vp]),
    "pgw_ev_row": (i32, [i32]),
    "pgw_agent_reduce": (i32, [P(ReduceArgs), i64, vp, vp, vp]),
    "pgw_pf_solve": (i32, [P(PFParams), P(PFTables), i64, vp, vp, vp, vp, vp]),
    "pgw_pf_solve_f32": (i32, [P(PFParams), P(PFTables), i64, vp, vp, vp, vp, vp]),
    "pgw_pf_solve_general": (i32, [P(PFGParams), P(PFGTables), i64, vp, vp, vp, vp, vp]),
    "pgw_reg_factor": (i32, [P(RegParams), i64, vp, vp, vp, vp]),
    "pgw_reg_control": (i32, [P(RegParams), i64, vp, vp, vp, vp, vp, vp]),
    "pgw_pf_padded_m": (i32, [i32]),
    "pgw_voltage_band_penalty": (i32, [i64, vp, f64, f64, f64, vp, vp]),
    "pgw_pf_pack_size": (i64, [i32]),
    "pgw_timing_start": (i32, [i32]),
    "pgw_debug_pf_trace": (i32, [vp]),
    "pgw_debug_mc_trace": (i32, [vp]),
    "pgw_pf_pred_meta": (i32, [P(PFParams), i32, i32, vp, vp, vp, vp]),
    "pgw_pf_pred_pack": (i32, [P(PFParams), i32, i32, vp, vp, vp]),
    "pgw_timing_stop": (i32, [vp, vp]),
    "pgw_stream_copy": (i32, [vp, vp, i64, i32, P(C.c_float), vp]),
    "pgw_pf_pack": (i32, [P(PFParams), vp, vp, vp, vp, vp]),
    "pgw_feeder_build": (i32, [P(FeederElem), i32, i32, vp, vp, vp, vp]),
    "pgw_pf_reduce": (i32, [i32, vp, vp, i32, vp, vp, i32, vp, vp, vp, vp, vp]),
    "pgw_coord_step": (i32, [P(CoordParams), P(PFParams), P(PFTables), P(CoordStepInfo), i64,
                             CoordBuffers, vp]),
    "pgw_coord_step_f32": (i32, [P(CoordParams), P(PFParams), P(PFTables), P(CoordStepInfo), i64,
                                 CoordBuffersF32, vp]),
    "pgw_coord_step_general": (i32, [P(CoordParams), P(PFGParams), P(PFGTables), P(CoordStepInfo), i64,
                                     CoordBuffers, vp]),
    "pgw_hs_reset": (i32, [P(HSParams), P(HSStepInfo), i64, vp, HSBuffers, vp]),
    "pgw_mc_agent_step": (i32, [P(MCStepArgs), i64, vp]),
    "pgw_mc_agent_step_f32": (i32, [P(MCStepArgsF32), i64, vp]),
    "pgw_mc_ev_split_mode": (i32, [i32, P(i32)]),
    "pgw_graph_begin": (i32, [vp]),
    "pgw_graph_end": (i32, [vp, P(vp)]),
    "pgw_graph_launch": (i32, [vp, vp]),
    "pgw_graph_destroy": (i32, [vp]),
    "pgw_hs_step": (i32, [P(HSParams), P(HSStepInfo), i64, HSBuffers, vp]),
    "pgw_ma_step": (i32, [P(MAStepArgs), P(PFParams), P(PFTables), i64, vp, vp, vp]),
}

EXPORTED = sorted(_SIGS)

STRUCTS = [Mat, BatteryParams, PVParams, BuildingParams, BuildingExo, BuildingExt, EVParams,
           EVStepInfo, ReduceArgs, PFParams, PFTables, FeederElem, CoordParams, CoordBuffers,
           CoordStepInfo, PredMeta, HSParams, HSStepInfo, HSBuffers, MCStepArgs, Matf, CoordBuffersF32,
           MAStepArgs, PFGElem, PFGParams, PFGTables, RegParams, MCStepDyn, PFOD, MCStepArgsF32]

_lib = None


def lib():
    """Load libpgw.so (once).  Raises PgwError if it is missing or mismatched."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PgwError("libpgw.so not found at %s -- build it with "
                       "`python -c 'import __graft_entry__ as g; g.build()'` or "
                       "`make -C powergridworld_amd/csrc`" % LIB_PATH)
    h = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(h, name)
        fn.restype = res
        fn.argtypes = args
    if h.pgw_abi_version() != ABI_VERSION:
        raise PgwError("libpgw ABI %d != expected %d (rebuild)" % (h.pgw_abi_version(), ABI_VERSION))
    sizes = (i64 * len(STRUCTS))()
    h.pgw_struct_sizes(sizes, len(STRUCTS))
    for st, sz in zip(STRUCTS, sizes):
        if C.sizeof(st) != sz:
            raise PgwError("ABI struct %s: ctypes %d B != C %d B" % (st.__name__, C.sizeof(st), sz))
    _lib = h
    return h


def check(rc):
    if rc != 0:
        raise PgwError(lib().pgw_last_error().decode() or ("libpgw error %d" % rc))


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device=None):
    """hipStream_t of torch's current stream on `device` (the raw accessor skips
    building a torch Stream object: this runs several times per env step)."""
    if _raw_stream is not None:
        idx = device.index if isinstance(device, torch.device) and device.index is not None else \
            (device if isinstance(device, int) else torch.cuda.current_device())
        return C.c_void_p(_raw_stream(idx))
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def dptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else C.c_void_p(t.data_ptr())


def mat(t2d):
    """pgw_mat for a 2-D [n_envs, dim] fp64 device tensor (any strides)."""
    if t2d is None:
        return Mat(None, 0, 0)
    assert t2d.dim() == 2 and t2d.dtype == torch.float64, (t2d.shape, t2d.dtype)
    return Mat(t2d.data_ptr(), t2d.stride(0), t2d.stride(1))


def matf(t2d):
    """pgw_matf for a 2-D [n_envs, dim] fp32 device tensor (any strides)."""
    if t2d is None:
        return Matf(None, 0, 0)
    assert t2d.dim() == 2 and t2d.dtype == torch.float32, (t2d.shape, t2d.dtype)
    return Matf(t2d.data_ptr(), t2d.stride(0), t2d.stride(1))


STORAGE_DTYPES = (torch.float64, torch.float32)


def storage_dtype(dtype):
    """The storage dtype of an env (fp64 = the reference's; fp32 = the _f32 entries)."""
    dtype = torch.float64 if dtype is None else dtype
    if dtype not in STORAGE_DTYPES:
        raise PgwError("storage dtype must be torch.float64 or torch.float32, got %s" % (dtype,))
    return dtype


def require_device(device):
    device = torch.device(device) if device is not None else torch.device("cuda")
    if device.type != "cuda":
        raise PgwError("powergridworld_amd runs its step kernels on the GPU only "
                       "(got device=%s); there is no CPU fallback" % device)
    if not torch.cuda.is_available():
        raise PgwError("no ROCm GPU visible: the HIP step kernels cannot run here")
    lib()
    return device
