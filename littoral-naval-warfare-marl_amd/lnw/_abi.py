"""ctypes binding of liblnw.so (include/lnw.h).

The product path: every call goes to the HIP library built in-tree for gfx950.
There is no CPU fallback — if the library is missing or fails to load, the
import raises.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liblnw.so")

LNW_SMALL, LNW_LARGE, LNW_LS, LNW_MEDIUM = 0, 1, 2, 3
LNW_ACT_F32, LNW_ACT_F64, LNW_ACT_I32 = 0, 1, 2
LNW_KIND_PYFLOAT, LNW_KIND_F32, LNW_KIND_F64 = 1, 2, 3
LNW_RNG_PHILOX, LNW_RNG_TAPE = 0, 1
LNW_OBS_ALL, LNW_OBS_BLUE, LNW_OBS_RED = -1, -2, -3
LNW_ERRF_ZERODIV, LNW_ERRF_NAN_ROUND, LNW_ERRF_TAPE, LNW_ERRF_MISSILES = 1, 2, 4, 8

(F_POS, F_RADAR, F_MISSILES, F_MKIND, F_ALIVE, F_TYPE, F_STEPS, F_DIST_LZ, F_TL_CNT, F_TL,
 F_DUCT, F_ENV, F_RNG, F_ERR) = range(14)
LNW_NFIELDS = 14

# exported symbols (must match include/lnw.h)
SYMBOLS = [
    "lnw_abi_version", "lnw_last_error", "lnw_create", "lnw_destroy", "lnw_load_terrain",
    "lnw_set_rng", "lnw_reset", "lnw_step", "lnw_step_seq", "lnw_observe", "lnw_observe_ex", "lnw_state_field", "lnw_tlist_cap",
    "lnw_set_epw", "lnw_set_variant", "lnw_set_reward_dtype",
    "lnw_set_counters",
    "lnw_los_batch", "lnw_astar_batch", "lnw_move_batch", "lnw_path_query", "lnw_los_query", "lnw_copy",
    "lnw_fill_uniform_f32", "lnw_hit_tables", "lnw_set_analytics", "lnw_actor_features",
    "lnw_state_bytes", "lnw_get_state", "lnw_set_state", "lnw_step_kernel",
    "lnw_policy_act", "lnw_rollout_post",
]

# lnw_step_kernel codes (include/lnw.h LNW_KERNEL_*)
(KERNEL_NONE, KERNEL_GENERIC, KERNEL_TEAM, KERNEL_TEAM_CONTACT, KERNEL_UNITS, KERNEL_GROUP,
 KERNEL_REFLOS) = range(7)


class Analytics(C.Structure):  # include/lnw.h: lnw_analytics
    _fields_ = [("heatmap", C.c_void_p), ("coldmap", C.c_void_p), ("launch", C.c_void_p),
                ("eng_log", C.c_void_p), ("eng_count", C.c_void_p), ("eng_cap", C.c_int64),
                ("ew_log", C.c_void_p), ("ew_count", C.c_void_p), ("ew_cap", C.c_int64)]


class Params(C.Structure):
    _fields_ = [("discrete", C.c_int32), ("landing_ops", C.c_int32), ("aggressive", C.c_int32),
                ("side_blue", C.c_int32), ("trained_red", C.c_int32), ("move_thr", C.c_int32),
                ("ew_thr", C.c_int32), ("lz_x", C.c_int32), ("lz_y", C.c_int32),
                ("red_aggression", C.c_double), ("episode_steps", C.c_int32),
                ("auto_reset", C.c_int32), ("los_mode", C.c_int32), ("move_mode", C.c_int32)]


class Spawn(C.Structure):
    _fields_ = [("types", C.c_int32 * 64), ("pos", (C.c_int32 * 2) * 64),
                ("rand_ls", C.c_int32 * 64), ("box_lo", C.c_int32 * 2),
                ("box_hi", C.c_int32 * 2)]


class Seq(C.Structure):  # include/lnw.h: lnw_seq
    _fields_ = [("steps", C.c_int32), ("act_step", C.c_int64), ("kind_step", C.c_int64),
                ("obs_blue_step", C.c_int64), ("obs_red_step", C.c_int64), ("rew_blue_step", C.c_int64),
                ("rew_red_step", C.c_int64), ("done_step", C.c_int64), ("cog_step", C.c_int64)]


class PolicyArgs(C.Structure):  # include/lnw.h: lnw_policy_args
    _fields_ = [("obs", C.c_void_p), ("E", C.c_int64),
                ("n", C.c_int32), ("D", C.c_int32), ("own0", C.c_int32), ("A", C.c_int32),
                ("params", C.c_void_p), ("bn_running", C.c_int32), ("forced", C.c_int32),
                ("forced_act", C.c_void_p), ("fa_env_stride", C.c_int64), ("noise", C.c_float),
                ("seed", C.c_uint64), ("call_dev", C.c_void_p),
                ("T", C.c_int32), ("t", C.c_int32), ("which", C.c_int32),
                ("row_base", C.c_int64), ("alive", C.c_void_p), ("live", C.c_void_p),
                ("obs_out", C.c_void_p), ("obs_env_stride", C.c_int64),
                ("act_out", C.c_void_p), ("logp_out", C.c_void_p), ("act_env_stride", C.c_int64),
                ("full", C.c_void_p), ("script", C.c_void_p),
                ("script_n", C.c_int32), ("script_steps", C.c_int32), ("script_own0", C.c_int32),
                ("script_cnt", C.c_int32), ("kinds", C.c_void_p), ("kinds_f32_all_alive", C.c_int32),
                ("f32_out", C.c_void_p), ("f32_env_stride", C.c_int64),
                ("obs_in_env_stride", C.c_int64)]


class RolloutPostArgs(C.Structure):  # include/lnw.h: lnw_rollout_post_args
    _fields_ = [("obs", C.c_void_p), ("obs_env_stride", C.c_int64), ("E", C.c_int64),
                ("n", C.c_int32), ("D", C.c_int32), ("critic", C.c_void_p), ("val", C.c_void_p),
                ("val_env_stride", C.c_int64), ("rew", C.c_void_p), ("rew_f64", C.c_int32),
                ("n_rew", C.c_int32), ("rew_out", C.c_void_p), ("rew_env_stride", C.c_int64),
                ("done", C.c_void_p), ("live", C.c_void_p), ("running", C.c_void_p),
                ("running_env_stride", C.c_int64), ("stop_at_done", C.c_int32)]


class LnwError(RuntimeError):
    pass


_lib = None


def load(path=None):
    """Load liblnw.so (raises if it is missing: no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("LNW_LIB", LIB_PATH)
    if not os.path.exists(path):
        raise LnwError(f"liblnw.so not built at {path}; run lnw.build.build() "
                       "(or __graft_entry__.build())")
    L = C.CDLL(path)
    P, I32, I64, U64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64
    sig = {
        "lnw_abi_version": ([], C.c_int),
        "lnw_last_error": ([], C.c_char_p),
        "lnw_create": ([C.POINTER(Params), I32, I32, I32, I32, I64, C.POINTER(P)], C.c_int),
        "lnw_destroy": ([P], C.c_int),
        "lnw_load_terrain": ([P, P, I32], C.c_int),
        "lnw_set_rng": ([P, I32, U64, P, P], C.c_int),
        "lnw_reset": ([P, P, C.POINTER(Spawn), P, P], C.c_int),
        "lnw_step": ([P, P, I32, P, P, P, P, P, P, P, P], C.c_int),
        "lnw_step_seq": ([P, C.POINTER(Seq), P, I32, P, P, P, P, P, P, P, P], C.c_int),
        "lnw_observe": ([P, I32, P, P, P], C.c_int),
        "lnw_observe_ex": ([P, I32, P, C.c_int64, P, C.c_int64, P], C.c_int),
        "lnw_state_field": ([P, I32, C.POINTER(P), C.POINTER(I64)], C.c_int),
        "lnw_tlist_cap": ([P], C.c_int),
        "lnw_set_epw": ([P, I32], C.c_int),
        "lnw_set_variant": ([P, I32], C.c_int),
        "lnw_set_reward_dtype": ([P, I32], C.c_int),
        "lnw_set_counters": ([P, P], C.c_int),
        "lnw_los_batch": ([P, I32, P, I64, I32, I32, P, P], C.c_int),
        "lnw_astar_batch": ([P, I32, I32, P, P, P, I64, P, P, P, P], C.c_int),
        "lnw_move_batch": ([P, P, P, P, P, I64, P, P, P], C.c_int),
        "lnw_path_query": ([P, P, P, P, I64, P, P], C.c_int),
        "lnw_los_query": ([P, P, I64, P, P], C.c_int),
        "lnw_copy": ([P, P, I64, P], C.c_int),
        "lnw_fill_uniform_f32": ([P, I64, U64, U64, P], C.c_int),
        "lnw_hit_tables": ([P, P], C.c_int),
        "lnw_set_analytics": ([P, P], C.c_int),
        "lnw_actor_features": ([P, I32, P, I64, I32, P, P], C.c_int),
        "lnw_state_bytes": ([P], C.c_int64),
        "lnw_get_state": ([P, P, I64, P], C.c_int),
        "lnw_set_state": ([P, P, I64, P], C.c_int),
        "lnw_step_kernel": ([P], C.c_int),
        "lnw_policy_act": ([C.POINTER(PolicyArgs), P], C.c_int),
        "lnw_rollout_post": ([C.POINTER(RolloutPostArgs), P], C.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def check(rc):
    if rc != 0:
        msg = _lib.lnw_last_error().decode() if _lib is not None else "?"
        raise LnwError(f"lnw call failed ({rc}): {msg}")
    return rc
