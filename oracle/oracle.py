"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of oracle/liboracle.so.

The CPU restatement of the reference env step (see pmenv_oracle.c for the
file:line map onto zachramsey/pm-rl). Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg use it, always as the checker, never as the thing
measured or shipped.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_P = ctypes.c_void_p
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: python pm-rl_amd/build.py")
        from pmenv._abi import PmenvCfg  # same struct layout as include/pmenv.h
        lib = ctypes.CDLL(LIB_PATH)
        lib.or_create.restype = _P
        lib.or_create.argtypes = [ctypes.POINTER(PmenvCfg)]
        lib.or_destroy.argtypes = [_P]
        lib.or_reset.argtypes = [_P, _P, _P]
        lib.or_step.argtypes = [_P, _P, _P, _P, _P, _P, _P, _P]
        lib.or_step_mt.argtypes = [_P, _P, _P, _P, _P, _P, _P, _P, ctypes.c_int]
        lib.or_gae.argtypes = [_P, _P, _P, _P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_float, ctypes.c_float]
        lib.or_moments.argtypes = [_P, ctypes.c_int64, _P]
        lib.or_philox4x32.argtypes = [ctypes.c_uint32] * 6 + [_P]
        lib.or_batch_reward.restype = ctypes.c_double
        lib.or_batch_reward.argtypes = [_P, _P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_double, _P, _P]
        lib.or_synth_series.argtypes = [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                        ctypes.c_uint64, ctypes.c_float]
        lib.or_synth_actions.argtypes = [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                         ctypes.c_uint64]
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(_P)


def _f32(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float32)


class _OrEnv(ctypes.Structure):
    pass


class OracleEnv:
    """Batched CPU env with the same reset/step contract as pmenv.TradingEnv."""

    def __init__(self, cfg):
        """cfg: pmenv.EnvConfig."""
        from pmenv._abi import PmenvCfg  # noqa: F401
        lib = load()
        self.cfg = cfg
        self._c = cfg.to_c()
        self._h = lib.or_create(ctypes.byref(self._c))
        B, N, W = cfg.num_envs, cfg.num_assets, cfg.window
        # struct or_env { pmenv_cfg cfg; double* value; int32_t* k; float* ring; double* sa; double* sb; }
        base = self._h + ctypes.sizeof(self._c)
        ptrs = (ctypes.c_void_p * 5).from_address(base)
        self.value = np.ctypeslib.as_array(ctypes.cast(ptrs[0], ctypes.POINTER(ctypes.c_double)), (B,))
        self.k = np.ctypeslib.as_array(ctypes.cast(ptrs[1], ctypes.POINTER(ctypes.c_int32)), (B,))
        self.ring = np.ctypeslib.as_array(ctypes.cast(ptrs[2], ctypes.POINTER(ctypes.c_float)), (B, W, N))
        self.stat_a = np.ctypeslib.as_array(ctypes.cast(ptrs[3], ctypes.POINTER(ctypes.c_double)), (B,))
        self.stat_b = np.ctypeslib.as_array(ctypes.cast(ptrs[4], ctypes.POINTER(ctypes.c_double)), (B,))

    def reset(self, obs=None, mask=None):
        """obs: float32 C-contiguous [B, N, W, F] numpy array, written in place."""
        if obs is not None:
            assert obs.dtype == np.float32 and obs.flags.c_contiguous
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        load().or_reset(self._h, _p(obs), _p(m))
        return obs

    def step(self, action, obs=None, prices=None, bar=None, threads=1):
        B, N = self.cfg.num_envs, self.cfg.num_assets
        a = _f32(action).reshape(B, N)
        p = None if prices is None else _f32(prices).reshape(B, N)
        br = None if bar is None else _f32(bar).reshape(B, N, self.cfg.features - 1)
        if obs is not None:
            assert obs.dtype == np.float32 and obs.flags.c_contiguous
        r = np.empty(B, np.float32)
        ret = np.empty(B, np.float64)
        w = np.empty((B, N), np.float32)
        load().or_step_mt(self._h, _p(a), _p(p), _p(br), _p(obs), _p(r), _p(ret), _p(w), int(threads))
        return r, ret, w

    def close(self):
        if self._h:
            load().or_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def gae(rewards, values, dones=None, gamma=0.99, lam=0.95):
    r = _f32(rewards)
    v = _f32(values)
    T, B = r.shape
    d = None if dones is None else np.ascontiguousarray(dones, dtype=np.uint8)
    adv = np.empty_like(r)
    ret = np.empty_like(r)
    load().or_gae(_p(r), _p(v), _p(d), _p(adv), _p(ret), T, B, gamma, lam)
    return adv, ret


def moments(x):
    x = _f32(x).reshape(-1)
    out = np.empty(3, np.float64)
    load().or_moments(_p(x), x.size, _p(out))
    return out


def philox4x32(ctr, key):
    out = np.empty(4, np.uint32)
    load().or_philox4x32(*[int(c) for c in ctr], *[int(k) for k in key], _p(out))
    return out


def synth_series(T, B, N, env_offset=0, seed=42, sigma=0.015):
    out = np.empty((T, B, N, 4), np.float32)
    load().or_synth_series(_p(out), T, B, N, env_offset, seed, sigma)
    return out


def synth_actions(T, B, N, env_offset=0, seed=43):
    out = np.empty((T, B, N), np.float32)
    load().or_synth_actions(_p(out), T, B, N, env_offset, seed)
    return out


BATCH_REWARD_KINDS = {"log_returns": 0, "returns": 1, "sharpe_ratio": 2}
BATCH_NORMS = {"global_or": 0, "row_or": 1, "none": 2}


def batch_reward(a, v_prev, p, reward="log_returns", norm="global_or", scale=1.0):
    """agent/pg/pg.py:40-82 restated: returns (R, ret [B], dR/da [B, N])."""
    a = _f32(a)
    B = a.shape[0]
    a = a.reshape(B, -1)
    N = a.shape[1]
    v = _f32(v_prev).reshape(B)
    pp = _f32(p).reshape(B, N)
    ret = np.empty(B, np.float32)
    grad = np.empty((B, N), np.float32)
    R = load().or_batch_reward(_p(a), _p(v), _p(pp), B, N, BATCH_REWARD_KINDS[reward], BATCH_NORMS[norm],
                               float(scale), _p(ret), _p(grad))
    return R, ret, grad


def replay_gather(series, days, actions, rewards, h0, env, W):
    """replay/buffer.py:53-79 restated in numpy for a ring of recorded steps."""
    T, N, Fm = series.shape
    H = days.shape[0]
    S = len(h0)
    s = np.empty((S, N, W, Fm + 1), np.float32)
    s2 = np.empty_like(s)
    a = np.empty((S, N), np.float32)
    r = np.empty(S, np.float32)
    for j in range(S):
        b, h = int(env[j]), int(h0[j])
        hist = np.stack([actions[(h + t) % H, b] for t in range(W + 1)], 1)      # [N, W+1]  (:59, :62)
        d = int(days[(h + W - 1) % H, b])                                           # (:65)
        for dd, out, ch in ((d, s, hist[:, :-1]), (d + 1, s2, hist[:, 1:])):        # (:66-70)
            for t in range(W):
                day = dd - (W - 1) + t
                out[j, :, t, :Fm] = series[day] if 0 <= day < T else np.nan
            out[j, :, :, Fm] = ch
        a[j] = hist[:, -1]                                                           # (:72)
        r[j] = rewards[(h + W - 1) % H, b]                                           # (:60)
    return s, a, r, s2


def trajectory_metrics(returns, values, weights, rf=0.04, periods=252):
    """util/eval.py:14-37 with quantstats' published formulas (sharpe, sortino,
    max_drawdown) and the reference's turnover loop, per env column."""
    returns = np.asarray(returns, np.float64)
    values = np.asarray(values, np.float64)
    weights = np.asarray(weights, np.float64)
    rfp = (1 + rf) ** (1 / periods) - 1 if rf else 0.0
    x = returns - rfp
    T = x.shape[0]
    sharpe = x.mean(0) / x.std(0, ddof=1) * np.sqrt(periods)
    sortino = x.mean(0) / np.sqrt((np.minimum(x, 0) ** 2).sum(0) / T) * np.sqrt(periods)
    mdd = (values / np.maximum.accumulate(values, 0) - 1).min(0)
    turn = np.abs(np.diff(weights, axis=0)).sum((0, 2)) / T
    return np.stack([sharpe, sortino, np.minimum(mdd, 0.0), turn, values[-1]], 1)
