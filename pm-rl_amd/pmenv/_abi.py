"""ctypes binding of include/pmenv.h (libpmenv.so, built in place for gfx950).

The product path has no CPU fallback: if libpmenv.so is missing or the HIP
runtime cannot load it, importing this module raises.
"""
import ctypes
import os

# torch must be imported first so libpmenv.so binds to the HIP runtime torch
# already loaded (same soname libamdhip64.so.7 -> one runtime, one device context).
import torch  # noqa: F401

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PMENV_LIB", os.path.join(HERE, "libpmenv.so"))

PMENV_ABI_VERSION = 3   # 2: pmenv_window_written / pmenv_state_written; cfg default ret_mode GROSS
                        # 3: pmenv_step_host / pmenv_reset_host

# enums (include/pmenv.h)
REWARD_KINDS = {"log_returns": 0, "returns": 1, "sharpe_ratio": 2, "diff_sharpe": 3}
NORM_MODES = {"and": 0, "or": 1}
RING_MODES = {"storage": 0, "chrono": 1}
RET_MODES = {"gross": 0, "net": 1, "auto": 2}
BATCH_NORM_MODES = {"global_or": 0, "row_or": 1, "none": 2}
STATE_FIELDS = 8   # value, stat_a, stat_b, counter, ring, nonfinite, last_close, w_new
STATUS = {0: "OK", -1: "ERR_ARG", -2: "ERR_SHAPE", -3: "ERR_HIP", -4: "ERR_ALIGN"}


class PmenvCfg(ctypes.Structure):
    _fields_ = [
        ("num_envs", ctypes.c_int32), ("num_assets", ctypes.c_int32), ("window", ctypes.c_int32),
        ("features", ctypes.c_int32), ("close_channel", ctypes.c_int32), ("reward_kind", ctypes.c_int32),
        ("norm_mode", ctypes.c_int32), ("ring_mode", ctypes.c_int32), ("ret_mode", ctypes.c_int32),
        ("mu_max_iter", ctypes.c_int32), ("init_cash", ctypes.c_double), ("commission", ctypes.c_double),
        ("reward_scale", ctypes.c_double), ("risk_free_rate", ctypes.c_double), ("sharpe_eta", ctypes.c_double),
        ("mu_tol", ctypes.c_double),
    ]


class PmenvStepArgs(ctypes.Structure):
    _fields_ = [
        ("action", ctypes.c_void_p), ("prices", ctypes.c_void_p), ("bar", ctypes.c_void_p),
        ("day", ctypes.c_void_p), ("series_days", ctypes.c_int32),
        ("obs", ctypes.c_void_p), ("obs_out", ctypes.c_void_p), ("reward", ctypes.c_void_p),
        ("ret", ctypes.c_void_p), ("weights", ctypes.c_void_p), ("phases", ctypes.c_uint32),
    ]


PHASE_SCALAR = 1
PHASE_ADVANCE = 2
STEP_PATHS = {"auto": 0, "one_launch": 1, "two_launch": 2, "flat": 3, "relay": 4}


# (name, restype, argtypes) for every symbol include/pmenv.h declares
_P = ctypes.c_void_p
_I32, _I64, _U64, _F, _SZ = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float, ctypes.c_size_t
SIGNATURES = [
    ("pmenv_cfg_default", None, [ctypes.POINTER(PmenvCfg), _I32, _I32, _I32, _I32]),
    ("pmenv_abi_version", _I32, []),
    ("pmenv_create", ctypes.c_int, [ctypes.POINTER(PmenvCfg), ctypes.c_int, ctypes.POINTER(_P)]),
    ("pmenv_state_bytes_for", _SZ, [ctypes.POINTER(PmenvCfg)]),
    ("pmenv_create_in", ctypes.c_int, [ctypes.POINTER(PmenvCfg), ctypes.c_int, _P, _SZ, ctypes.POINTER(_P)]),
    ("pmenv_state_layout", ctypes.c_int, [ctypes.POINTER(PmenvCfg), ctypes.POINTER(_SZ)]),
    ("pmenv_destroy", ctypes.c_int, [_P]),
    ("pmenv_last_error", ctypes.c_char_p, [_P]),
    ("pmenv_get_cfg", ctypes.c_int, [_P, ctypes.POINTER(PmenvCfg)]),
    ("pmenv_reset", ctypes.c_int, [_P, _P, _P, _P]),
    ("pmenv_step_ex", ctypes.c_int, [_P, ctypes.POINTER(PmenvStepArgs), _P]),
    ("pmenv_step", ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P]),
    ("pmenv_step_host", ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P]),
    ("pmenv_reset_host", ctypes.c_int, [_P, _P, _P, _P]),
    ("pmenv_value", _P, [_P]),
    ("pmenv_ring", _P, [_P]),
    ("pmenv_counter", _P, [_P]),
    ("pmenv_state_bytes", _SZ, [_P]),
    ("pmenv_step_path", ctypes.c_char_p, [_P]),
    ("pmenv_set_step_path", ctypes.c_int, [_P, _I32]),
    ("pmenv_window_written", ctypes.c_int, [_P, _P, _P]),
    ("pmenv_state_written", ctypes.c_int, [_P, _P]),
    ("pmenv_get_state", ctypes.c_int, [_P, _P, _P]),
    ("pmenv_set_state", ctypes.c_int, [_P, _P, _P]),
    ("pmenv_nonfinite_count", ctypes.c_int, [_P, ctypes.POINTER(_U64), _P]),
    ("pmenv_synth_series", ctypes.c_int, [_P, _I32, _I32, _I32, _I64, _U64, _F, _P]),
    ("pmenv_synth_actions", ctypes.c_int, [_P, _I32, _I32, _I32, _I64, _U64, _P]),
    ("pmenv_window_init", ctypes.c_int, [_P, _P, _I32, _I32, _I32, _I32, _P]),
    ("pmenv_window_init_days", ctypes.c_int, [_P, _P, _I32, _I32, _I32, _P, _I32, _I32, _P]),
    ("pmenv_gae", ctypes.c_int, [_P, _P, _P, _P, _P, _I32, _I32, _F, _F, _P]),
    ("pmenv_gae_workspace", _SZ, [_I32, _I32]),
    ("pmenv_gae_ex", ctypes.c_int, [_P, _P, _P, _P, _P, _I32, _I32, _F, _F, _P, _SZ, _P]),
    ("pmenv_moments_workspace", ctypes.c_size_t, []),
    ("pmenv_moments", ctypes.c_int, [_P, _I64, _P, _P, _P]),
    ("pmenv_replay_gather", ctypes.c_int,
     [_P, _I32, _I32, _I32, _I32, _P, _P, _P, _I32, _I32, _P, _P, _I32, _P, _P, _P, _P, _P]),
    ("pmenv_rollout_gather", ctypes.c_int,
     [_P, _I32, _I32, _I32, _I32, _P, _P, _I32, _I32, _I32, _P, _P, _I32, _P, _P]),
    ("pmenv_metrics", ctypes.c_int, [_P, _P, _P, _I32, _I32, _I32, ctypes.c_double, ctypes.c_double, _P, _P]),
    ("pmenv_batch_reward_workspace", _SZ, [_I32]),
    ("pmenv_batch_reward_forward", ctypes.c_int,
     [_P, _P, _P, _I32, _I32, _I32, _I32, ctypes.c_double, _P, _P, _P, _P]),
    ("pmenv_batch_reward_backward", ctypes.c_int,
     [_P, _P, _P, _I32, _I32, _I32, ctypes.c_double, _P, _P, _P, _P]),
]

_lib = None


def load():
    """Load libpmenv.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not found: build it with `python pm-rl_amd/build.py` "
                          "(or __graft_entry__.build()); pmenv has no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    # the version first: a stale library fails here, not on a symbol it does not export
    ver = getattr(lib, "pmenv_abi_version", None)
    if ver is None:
        raise ImportError(f"{LIB_PATH} exports no pmenv_abi_version: not a libpmenv build")
    ver.restype, ver.argtypes = ctypes.c_int32, []
    if ver() != PMENV_ABI_VERSION:
        raise ImportError(f"libpmenv ABI {ver()} != {PMENV_ABI_VERSION}: rebuild with `python pm-rl_amd/build.py`")
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class PmenvError(RuntimeError):
    pass


def check(rc, handle=None, what="pmenv"):
    if rc != 0:
        msg = load().pmenv_last_error(handle)
        raise PmenvError(f"{what} failed ({STATUS.get(rc, rc)}): {msg.decode() if msg else ''}")
