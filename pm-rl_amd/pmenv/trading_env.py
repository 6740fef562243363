"""TradingEnv — batched, device-resident drop-in for the reference env.

Mirrors zachramsey/pm-rl env/sim/trading_env.py (`TradingEnv`, :7-115) call for
call, with a leading batch dimension B of lockstep envs:

    reference                                  here
    TradingEnv()                      :8-18    TradingEnv()  (shape bound by the first reset / step)
                                               TradingEnv(num_envs=B, num_assets=N, window=W, features=F)
    reset(features) -> features       :21-41   reset(features[, mask]) -> features  (in place)
    step(action, features, prices)    :44-105  step(action, features, prices) -> (r, features)
      -> (r, features)                         step(action, features, bar=bar)  (fused window advance)
    .value                            :9,89    .value  (f64 [B], device view; host 0-dim with host I/O)
    .weights (ActionBuffer)           :10      .weights (RingView: get_last / get_all)
    .info values/actions/rewards/returns       .info (kept by default for one env, as the reference)

`TradingEnv()` with no arguments is the reference's constructor (`train/on_policy.py:35`):
the reference sizes its ring from config/base.py's NUM_ASSETS / WINDOW_SIZE and takes
whatever feature count the data pool carries (`data/data_loader.py:48`), so here every
dimension that is not given — envs, assets, window, features — is taken from the first
`reset(features)` (or `step`) tensor: `[N, W, F]` for one env, `[B, N, W, F]` for B.
Dimensions that are given are checked against it (ValueError, as a ring of the wrong
shape fails in the reference). `info` is kept by default when the env holds one env
(the reference always keeps it, :13-18, :34-39); pass `track_info=` to choose.

Every compute call goes through libpmenv.so (include/pmenv.h); there is no CPU
path. `features` must be a float32, contiguous tensor: it is written in place and
returned, exactly as trading_env.py:32,103 mutate the caller's tensor. A caller that
keeps the reference's CPU tensors (train/on_policy.py:59-67 hands the env host
tensors) may pass them unchanged: reset / step (surface contract) then run through
pmenv_reset_host / pmenv_step_host — only the action, the prices and the window's last
closes go to the GPU, only the [N, W] weight channel and the outputs come back, through
pinned device-mapped staging with one stream sync per call — and the reward, `.value`
and `.info` are host objects with the reference's types. (The fused advance with host
tensors stages the whole window to the GPU and back; keep tensors on the GPU for
throughput.)
"""
import ctypes
import weakref

import numpy as np
import torch

from . import _abi
from .config import EnvConfig, NUM_ASSETS, WINDOW_SIZE

_CPU = torch.device("cpu")


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
if _raw_stream is None:                        # older torch: the public (slower) accessor
    def _raw_stream(index):
        return torch.cuda.current_stream(index).cuda_stream


def _version(t):
    """t's in-place write counter; None for inference-mode tensors, which keep none
    (their edits are then assumed on every step)."""
    try:
        return t._version
    except RuntimeError:
        return None


class RingView:
    """Read-only view of the device weight ring with ActionBuffer's accessors
    (env/sim/weight_buffer.py:28-44); for inspection and tests, not the hot path."""

    def __init__(self, env):
        self._env = env

    @property
    def buffer(self):                      # [B, W, N] (weight_buffer.py:8)
        return self._env._ring

    @property
    def idx(self):                         # [B] (weight_buffer.py:10,22)
        return (1 + self._env._counter.long()) % self._env.cfg.window

    @property
    def is_full(self):                     # [B] (weight_buffer.py:11,25-26)
        return self._env._counter.long() >= self._env.cfg.window - 1

    def get_last(self):                    # [B, N] (weight_buffer.py:28-30)
        W = self._env.cfg.window
        k = self._env._counter.long() % W
        return self._env._ring[torch.arange(k.numel(), device=k.device), k]

    def get_all(self):                     # [B, N, W] (weight_buffer.py:32-44)
        cfg = self._env.cfg
        W = cfg.window
        ring = self._env._ring                                     # [B, W, N]
        B = ring.shape[0]
        idx = self.idx.view(B, 1)
        t = torch.arange(W, device=ring.device).view(1, W)
        pad = W - idx
        pre = t - pad                                               # not full: zero pad then ring[:idx]
        if cfg.ring == "storage":
            full_slot = t.expand(B, W)
        else:
            full_slot = (idx + t) % W
        slot = torch.where(self.is_full.view(B, 1), full_slot, pre.clamp(min=0))
        vals = torch.gather(ring, 1, slot.unsqueeze(-1).expand(B, W, ring.shape[2]))
        vals = torch.where((~self.is_full.view(B, 1, 1)) & (pre.unsqueeze(-1) < 0), torch.zeros_like(vals), vals)
        return vals.transpose(1, 2)


class TradingEnv:
    _DIMS = ("num_envs", "num_assets", "window", "features")

    def __init__(self, num_envs=None, num_assets=None, window=None, features=None, device=None,
                 config=None, track_info=None, step_impl="auto", **overrides):
        """step_impl: "auto" (per shape), "one_launch" (step_env_kernel, one workgroup per
        env), "flat" (step_flat_kernel, one launch over 16 KiB window tiles) or
        "two_launch" (scalar-step kernel + window stream); see set_step_impl.
        Dimensions left as None are bound by the first reset / step tensor (until then
        the handle holds config/base.py's shape: one env, 32 assets, window 32, F = 5).
        track_info: None keeps `info` when the env holds one env (the reference's case)."""
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("pmenv runs on a GPU device only (no CPU fallback)")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self._lib = _abi.load()
        given = dict(num_envs=num_envs, num_assets=num_assets, window=window, features=features)
        self._given = given
        if config is None:
            self._free = {k for k, v in given.items() if v is None}     # bound by the first tensor
            self._overrides = dict(overrides)
            config = self._config(dict(num_envs=1, num_assets=NUM_ASSETS, window=WINDOW_SIZE, features=5))
        else:
            self._free = set()
            self._overrides = {}
        self._track_info_arg = track_info
        self.step_impl = step_impl
        self._h = None
        self._build(config)

    def _config(self, dims):
        """EnvConfig of the given dims with the constructor's explicit values and overrides;
        a close channel not given is the OHLC close (3), or the last market channel below F = 5."""
        kw = {k: (self._given[k] if self._given[k] is not None else dims[k]) for k in self._DIMS}
        kw.update(self._overrides)
        if "close_channel" not in self._overrides:
            kw["close_channel"] = min(3, kw["features"] - 2)
        return EnvConfig(**kw)

    def _build(self, config):
        """Create the handle (and its state views) for `config`."""
        self.cfg = config.validate()
        self._c = self.cfg.to_c()
        nbytes = self._lib.pmenv_state_bytes_for(ctypes.byref(self._c))
        if nbytes == 0:
            raise ValueError("invalid env shape")
        off = (ctypes.c_size_t * _abi.STATE_FIELDS)()
        _abi.check(self._lib.pmenv_state_layout(ctypes.byref(self._c), off), None, "pmenv_state_layout")
        with torch.inference_mode(False):      # a normal tensor: its views count in-place writes
            self._state = torch.zeros(nbytes, dtype=torch.uint8, device=self.device)
        h = ctypes.c_void_p()
        torch.cuda.synchronize(self.device)
        _abi.check(self._lib.pmenv_create_in(ctypes.byref(self._c), self.device.index, _ptr(self._state),
                                             nbytes, ctypes.byref(h)), None, "pmenv_create_in")
        self._h = h
        B, N, W = self.cfg.num_envs, self.cfg.num_assets, self.cfg.window
        s = self._state
        with torch.inference_mode(False):
            self._value = s[off[0]:off[0] + 8 * B].view(torch.float64)
            self._stat_a = s[off[1]:off[1] + 8 * B].view(torch.float64)
            self._stat_b = s[off[2]:off[2] + 8 * B].view(torch.float64)
            self._counter = s[off[3]:off[3] + 4 * B].view(torch.int32)
            self._ring = s[off[4]:off[4] + 4 * B * W * N].view(torch.float32).view(B, W, N)
            self._nonfinite = s[off[5]:off[5] + 8].view(torch.int64)
            self._last_close = s[off[6]:off[6] + 4 * B * N].view(torch.float32).view(B, N)
            self._w_new = s[off[7]:off[7] + 4 * B * N].view(torch.float32).view(B, N)
        self.weights = RingView(self)
        self._obs_shape = (B, N, W, self.cfg.features)
        self._obs_size = torch.Size(self._obs_shape)
        self._obs_size_unb = torch.Size(self._obs_shape[1:]) if B == 1 else None
        self._bn = B * N
        self._dev_index = self.device.index
        self._args = _abi.PmenvStepArgs()          # reused: every field is set on every step
        self.track_info = (B == 1) if self._track_info_arg is None else bool(self._track_info_arg)
        # the last reset/step came unbatched / with CPU tensors; a TradingEnv() whose shape
        # the first call binds looks like the reference's (host, one env) until then
        self._unbatched = self._host_io = bool(self._free) and B == 1
        # caller edits between steps (trading_env.py:102-105: the features are the caller's):
        # the version counters of the state blob (shared by .value and every other view)
        # and of the last in-place window, as this wrapper left them; a change tells the
        # handle to re-read what its one-launch step keeps from the previous step
        self._state_ver = _version(self._state)
        self._win = None
        self._win_ver = -1
        # host I/O: the per-call record chunks and the host value of the last host-I/O call
        # (valid while the state blob is as that call left it)
        self._rec_blk, self._rec_n, self._rec_i = None, 0, 0
        self._hval, self._hval_ver = None, None
        self.set_step_impl(self.step_impl)
        self._reset_info()

    def _fit(self, features):
        """Bind the dimensions the constructor left open to the first tensor the env sees
        (trading_env.py sizes nothing itself: config/base.py and the data pool do)."""
        if not self._free:
            return
        shape = tuple(features.shape)
        if len(shape) == 4:
            dims = dict(zip(self._DIMS, shape))
        elif len(shape) == 3:
            dims = dict(zip(self._DIMS[1:], shape), num_envs=1)
        else:
            raise ValueError(f"features must be [N, W, F] or [B, N, W, F], got {shape}")
        self._free = set()
        cfg = self._config(dims)
        if tuple(getattr(cfg, k) for k in self._DIMS) != tuple(getattr(self.cfg, k) for k in self._DIMS) or \
                cfg.close_channel != self.cfg.close_channel:
            self.close()
            self._build(cfg)

    # ------------------------------------------------------------------ helpers
    def _stream(self):
        # the raw hipStream_t of the current stream (an int: ctypes passes it as void*)
        return _raw_stream(self._dev_index)

    def _reset_info(self):
        """trading_env.py:13-18 / :34-39 (dict order is relied on by util/plot.py:61). With
        host I/O and one env the entries have the reference's types: the seed entries are
        Python 0s, INITIAL_CASH and the all-cash get_last() tensor; each step appends the
        value as a 0-dim tensor (:80) and w', the return and the reward as numpy arrays
        (:85, :90, :100; value and return in f64, the precision the env computes in).
        The seed action is, in the reference, a VIEW of ring slot 0 (get_last() returns
        `self.buffer[(idx - 1) % W]`, weight_buffer.py:28-30, and `.flatten()` of a 1-D
        view is that view, :36): once the ring wraps it shows the w' last written there. The host-typed
        seed entry follows it (refreshed from the device ring whenever `info` is read, and
        frozen at the next reset, as the reference's reset swaps in a new buffer)."""
        self._info = None
        self._pending = []
        self._slot0 = None
        if not self.track_info:
            return
        B, N = self.cfg.num_envs, self.cfg.num_assets
        if self._host_io and self._unbatched:
            e0 = torch.zeros(N)
            e0[0] = 1
            ic = self.cfg.init_cash
            self._info = {"values": [int(ic) if float(ic).is_integer() else ic], "actions": [e0],
                          "rewards": [0], "returns": [0]}
            self._slot0 = e0
            self._slot0_dirty = False
            return
        dev = _CPU if self._host_io else self.device
        e0 = torch.zeros(B, N, device=dev)
        e0[:, 0] = 1
        self._info = {"values": [self._value.to(dev, copy=True)], "actions": [e0],
                      "rewards": [torch.zeros(B, device=dev)],
                      "returns": [torch.zeros(B, device=dev, dtype=torch.float64)]}

    def _sync_slot0(self):
        """The host-typed seed action <- ring slot 0 of the env (the reference's alias)."""
        if self._slot0 is not None and self._slot0_dirty:
            self._slot0.copy_(self._ring[0, 0])
            self._slot0_dirty = False

    @property
    def info(self):
        """The reference's per-step history (values, actions, rewards, returns), or None when
        not tracked. Host-I/O records are copied to the host when `info` is read (one copy
        per array for all steps since the last read), not on every step."""
        if self._info is None:
            return None
        if self._pending:
            self._flush_info()
        self._sync_slot0()
        return self._info

    @info.setter
    def info(self, value):
        self._pending = []
        self._slot0 = None
        self._info = value

    def _flush_info(self):
        pend, self._pending = self._pending, []
        vals = torch.stack([p[0] for p in pend]).cpu()
        acts = torch.stack([p[1] for p in pend]).cpu().numpy()
        rets = torch.stack([p[2] for p in pend]).cpu().numpy()
        rews = torch.stack([p[3] for p in pend]).cpu().numpy()
        inf = self._info
        for i in range(len(pend)):
            if self._unbatched:
                inf["values"].append(vals[i, 0])
                inf["actions"].append(acts[i, 0])
                inf["returns"].append(rets[i, 0, ...])        # 0-dim arrays, as .cpu().numpy()
                inf["rewards"].append(rews[i, 0, ...])
            else:
                inf["values"].append(vals[i])
                inf["actions"].append(acts[i])
                inf["returns"].append(rets[i])
                inf["rewards"].append(rews[i])

    def _obs_check(self, features, name="features"):
        if features.shape == self._obs_size and features.dtype is torch.float32 and features.is_cuda and \
                features.get_device() == self._dev_index and features.is_contiguous():
            return False                                   # the common case: a batched device window
        cfg = self.cfg
        shape = self._obs_shape
        if features.dtype != torch.float32 or not features.is_contiguous() or \
                features.device not in (self.device, _CPU):
            raise ValueError(f"{name} must be a contiguous float32 tensor on {self.device} or the host "
                             "(written in place)")
        if tuple(features.shape) == shape:
            return False
        if cfg.num_envs == 1 and tuple(features.shape) == shape[1:]:
            return True
        raise ValueError(f"{name} must have shape {shape} (or {shape[1:]} when num_envs == 1), "
                         f"got {tuple(features.shape)}")

    def _vec(self, x, per_env, name):
        """Coerce an action / prices tensor to a contiguous float32 [B, per_env]."""
        B = self.cfg.num_envs
        if not torch.is_tensor(x):
            x = torch.as_tensor(x)
        elif x.dtype is torch.float32 and x.is_cuda and x.get_device() == self._dev_index and x.is_contiguous() \
                and x.numel() == B * per_env:
            return x                                # the common case: as is (only its data pointer is used)
        if x.numel() != B * per_env:
            # weight_buffer.py:18-19 raises ValueError on a mis-shaped action
            raise ValueError(f"{name} must have {B} x {per_env} elements, got shape {tuple(x.shape)}")
        return x.to(device=self.device, dtype=torch.float32).reshape(B, per_env).contiguous()

    # ------------------------------------------------------------------ API
    @property
    def value(self):
        """Portfolio value (trading_env.py:9,89) — f64 [B] view of the device state
        (a host copy when the caller drives the env with CPU tensors)."""
        if self._host_io:
            hv = self._hval
            if hv is not None and self._hval_ver == _version(self._state) and self._hval_ver is not None:
                return hv                          # the host copy the last host-I/O call left
            v = self._value.cpu()
        else:
            v = self._value
        return v[0] if self._unbatched else v

    def set_step_impl(self, impl):
        """Advance-mode step implementation (pmenv_set_step_path): "auto", "one_launch",
        "flat" or "two_launch". Raises ValueError when the shape does not fit it."""
        if impl not in _abi.STEP_PATHS:
            raise ValueError(f"step_impl must be one of {sorted(_abi.STEP_PATHS)}")
        rc = self._lib.pmenv_set_step_path(self._h, _abi.STEP_PATHS[impl])
        if rc != 0:
            raise ValueError(self._lib.pmenv_last_error(self._h).decode())
        self.step_impl = impl

    @property
    def num_envs(self):
        return self.cfg.num_envs

    def reset(self, features=None, mask=None):
        """trading_env.py:21-41 for all envs (or the envs where mask is True)."""
        unb = False
        dev_features = features
        self._hval = None
        if features is not None:
            self._fit(features)
            unb = self._obs_check(features)
            self._unbatched = unb
            self._host_io = features.device.type == "cpu"
            if self._host_io and mask is None and self._HOST_DIRECT:   # the driver's reset (on_policy.py:61)
                if self._info is not None:
                    _ = self.info                  # the old history, final (flushed, seed action frozen)
                self._reset_host(features, unb)
                self._state_ver = _version(self._state)
                self._reset_info()
                return features
            if self._host_io:
                dev_features = features.to(self.device)
        if mask is None and self._info is not None:
            _ = self.info                     # the old history, final (flushed, seed action frozen)
        m = None
        if mask is not None:
            m = torch.as_tensor(mask).to(self.device).reshape(-1).to(torch.uint8).contiguous()
            if m.numel() != self.cfg.num_envs:
                raise ValueError("mask must have num_envs elements")
        _abi.check(self._lib.pmenv_reset(self._h, _ptr(dev_features), _ptr(m), self._stream()), self._h,
                   "pmenv_reset")
        if dev_features is not features:
            features.copy_(dev_features)
        self._state_ver = _version(self._state)
        if dev_features is not None:
            self._watch(dev_features)
        if mask is None:
            self._reset_info()
        return features

    def step(self, action, features, prices=None, bar=None, out=None, series=None, day=None, weights_out=None):
        """trading_env.py:44-105 for all B envs in one kernel launch.

        prices given, bar None : the reference contract — `features` is the next
                                 day's window; channel F-1 is rewritten in place.
        bar given              : fused path — `features` (the window returned by
                                 the previous reset/step) is advanced one day in
                                 place and `bar` [B, N, F-1] appended; prices
                                 default to bar.close / window[W-1].close.
        series, day            : resident data path — `series` is a pmenv.data.MarketSeries
                                 (or a [T, N, F-1] tensor) and env b takes day[b]'s
                                 bar from it (instead of `bar`)
        out (fused path only)  : write the advanced window into `out` instead of
                                 in place (double-buffered windows, as the
                                 reference's data path hands the env a fresh
                                 window every day); returns (r, out).
        weights_out            : a float32 [B, N] GPU tensor that receives the
                                 post-drift weights w' (info["actions"], :83-85)
        Returns (r, features); r is f32 [B] (0-dim for unbatched single-env input).

        Caller edits between fused in-place steps are honoured (the reference keeps no copy
        of the features): the wrapper compares torch's version counters of the window and
        of the state before each step. Writes those counters miss — `.data`, DLPack, raw
        kernels, or edits between replays of a captured hipGraph, where this check ran
        once at capture — must be announced with window_written(features) /
        state_written(), or the next flat step composes tile seams from stale copies.
        """
        if self._free:
            self._fit(features)
        if not features.is_cuda and bar is None and series is None and out is None and weights_out is None \
                and prices is not None and self._HOST_DIRECT:
            return self._step_host(action, features, prices)
        unb = self._obs_check(features)
        if not features.is_cuda:                    # the reference's CPU tensors: staged through the GPU
            if out is not None and out.device.type != "cpu":
                raise ValueError("out must live where features does")
            dev_out = None if out is None else torch.empty(out.shape, dtype=out.dtype, device=self.device)
            r, res = self._step(action, features.to(self.device), prices, bar, dev_out, series, day,
                                weights_out, unb, host=True)
            (features if out is None else out).copy_(res)
            self._host_io = True
            return r.cpu(), (features if out is None else out)
        if out is not None and not out.is_cuda:
            raise ValueError("out must live where features does")
        self._host_io = False
        return self._step(action, features, prices, bar, out, series, day, weights_out, unb, host=False)

    # ------------------------------------------------------------------ host I/O
    # The reference driver's call shape (train/on_policy.py:59-67): CPU action, window and
    # prices. One pmenv_step_host call per step: the kernel reads the action, the prices and
    # the window's last closes from pinned device-mapped staging and writes the [B, N, W]
    # weight channel back into it; the library scatters the channel into `features` (the
    # market channels never cross PCIe) and fills the per-step records below, so `.value`,
    # the reward and `info` need no further device round trip.
    _REC_STEPS = 256
    _HOST_DIRECT = True      # False: stage the whole window through the GPU (round 4's path; A/B only)

    def _host_vec(self, x, name):
        """action / prices as a host float32 contiguous tensor of B*N elements."""
        n = self._bn
        if type(x) is torch.Tensor and x.dtype is torch.float32 and not x.is_cuda and x.numel() == n \
                and x.is_contiguous():
            return x                                # the common case: as is (only its data pointer is used)
        if not torch.is_tensor(x):
            x = torch.as_tensor(x)
        if x.numel() != n:
            # weight_buffer.py:18-19 raises ValueError on a mis-shaped action
            raise ValueError(f"{name} must have {self.cfg.num_envs} x {self.cfg.num_assets} elements, "
                             f"got shape {tuple(x.shape)}")
        return x.detach().to(device=_CPU, dtype=torch.float32).contiguous()

    def _rec(self):
        """Host arrays for one call's outputs: views into chunks of _REC_STEPS calls, so a call
        costs no allocation and the records handed to the caller (the reward, `.value`,
        info entries) stay valid after later calls."""
        i = self._rec_i
        if self._rec_blk is None or i == self._rec_n:
            B, N = self.cfg.num_envs, self.cfg.num_assets
            K = max(1, min(self._REC_STEPS, (1 << 22) // (B * (N + 6) * 4)))
            blk = (np.empty((K, B), np.float32), np.empty((K, B), np.float64), np.empty((K, B), np.float64),
                   np.empty((K, B, N), np.float32))
            self._rec_blk, self._rec_n, i = blk, K, 0
            self._rec_ptr = tuple(a.ctypes.data for a in blk)
            self._rec_sz = (4 * B, 8 * B, 8 * B, 4 * B * N)
        self._rec_i = i + 1
        return i

    def _step_host(self, action, features, prices):
        shp = features.shape
        if shp == self._obs_size:
            unb = False
        elif shp == self._obs_size_unb:
            unb = True
        else:
            unb = self._obs_check(features)         # raises with the expected shapes
        if features.dtype is not torch.float32 or not features.is_contiguous():
            self._obs_check(features)               # raises
        a = self._host_vec(action, "action")
        p = self._host_vec(prices, "prices")
        track = self.track_info and self._info is not None
        i = self._rec()
        rp, sz = self._rec_ptr, self._rec_sz
        rc = self._lib.pmenv_step_host(self._h, a.data_ptr(), p.data_ptr(), features.data_ptr(), rp[0] + i * sz[0],
                                       rp[2] + i * sz[2], rp[1] + i * sz[1] if track else None,
                                       rp[3] + i * sz[3] if track else None, self._stream())
        if rc:
            _abi.check(rc, self._h, "pmenv_step_host")
        blk = self._rec_blk
        if unb:                                    # 0-dim / [N] entries, as the reference's .cpu().numpy()
            rew, ret, val, w = blk[0][i, 0, ...], blk[1][i, 0, ...], blk[2][i, 0, ...], blk[3][i, 0]
        else:
            rew, ret, val, w = blk[0][i], blk[1][i], blk[2][i], blk[3][i]
        r = torch.from_numpy(rew)                  # r and info["rewards"][-1] share memory, as :99-100
        v = torch.from_numpy(val)
        self._hval, self._hval_ver = v, _version(self._state)
        self._host_io = True
        self._unbatched = unb
        if track:
            if self._pending:
                self._flush_info()
            inf = self._info
            inf["values"].append(v)                # :80 the value tensor (also .value, :89)
            inf["actions"].append(w)               # :85 w'.cpu().numpy()
            inf["returns"].append(ret)             # :90
            inf["rewards"].append(rew)             # :100
            self._slot0_dirty = True
        return r, features

    def _reset_host(self, features, unb):
        i = self._rec()
        rp, sz = self._rec_ptr, self._rec_sz
        _abi.check(self._lib.pmenv_reset_host(self._h, features.data_ptr(), rp[2] + i * sz[2], self._stream()),
                   self._h, "pmenv_reset_host")
        val = self._rec_blk[2][i]
        self._hval, self._hval_ver = torch.from_numpy(val[0, ...] if unb else val), _version(self._state)

    def _step(self, action, features, prices, bar, out, series, day, weights_out, unb, host):
        self._hval = None
        cfg = self.cfg
        B, N = cfg.num_envs, cfg.num_assets
        a = self._vec(action, N, "action")
        p = self._vec(prices, N, "prices") if prices is not None else None
        br = dy = None
        days = 0
        if series is not None:
            sb = series.bars if hasattr(series, "bars") else series
            if sb.dim() != 3 or sb.shape[1] != N or sb.shape[2] != cfg.features - 1 or sb.dtype != torch.float32 \
                    or not sb.is_contiguous() or sb.device != self.device:
                raise ValueError(f"series must be a contiguous float32 [T, {N}, {cfg.features - 1}] on {self.device}")
            if day is None:
                raise ValueError("series= needs day= (one day index per env)")
            dy = torch.as_tensor(day, device=self.device).to(torch.int32).reshape(-1).contiguous()
            if dy.numel() != B:
                raise ValueError("day must hold one index per env")
            br, days = sb, sb.shape[0]
            bar = sb
        elif bar is not None:
            br = self._vec(bar, N * (cfg.features - 1), "bar")
        elif p is None:
            raise ValueError("step needs prices (reference contract) or bar (fused window advance)")
        r = torch.empty(B, dtype=torch.float32, device=self.device)
        args = self._args
        args.day, args.series_days, args.obs_out, args.ret, args.weights, args.phases = None, 0, None, None, None, 0
        args.action = a.data_ptr()
        args.prices = p.data_ptr() if p is not None else None
        args.bar = br.data_ptr() if br is not None else None
        if dy is not None:
            args.day = dy.data_ptr()
            args.series_days = days
        args.obs = features.data_ptr()
        if out is not None:
            if bar is None:
                raise ValueError("out= applies to the fused window advance (bar=...) only")
            if self._obs_check(out, "out") != unb:
                raise ValueError("out must have the same shape as features")
            args.obs_out = out.data_ptr()
        args.reward = r.data_ptr()
        stream = self._stream()
        self._edits(features if (br is not None and out is None) else None, stream)
        ret = w = None
        if weights_out is not None:
            if weights_out.dtype != torch.float32 or not weights_out.is_contiguous() or \
                    weights_out.device != self.device or weights_out.numel() != B * N:
                raise ValueError(f"weights_out must be a contiguous float32 [{B}, {N}] tensor on {self.device}")
            args.weights = weights_out.data_ptr()
        track = self.track_info and self._info is not None
        if track:
            ret = torch.empty(B, dtype=torch.float64, device=self.device)
            args.ret = ret.data_ptr()
            if weights_out is None:
                w = torch.empty(B, N, dtype=torch.float32, device=self.device)
                args.weights = w.data_ptr()
        _abi.check(self._lib.pmenv_step_ex(self._h, ctypes.byref(args), stream), self._h, "pmenv_step")
        if out is None and br is not None:
            self._watch(features)
        if track:
            # trading_env.py:80,85,90,100
            wv = w if weights_out is None else weights_out.reshape(B, N).clone()
            if host:
                self._pending.append((self._value.clone(), wv, ret, r))
                self._slot0_dirty = True
            else:
                self._info["values"].append(self._value.clone())
                self._info["actions"].append(wv)
                self._info["returns"].append(ret)
                self._info["rewards"].append(r)
        self._unbatched = unb
        return (r[0] if unb else r), (features if out is None else out)

    def _watch(self, window):
        """Remember the window as the handle left it (it is stepped in place next)."""
        self._win = weakref.ref(window)
        self._win_ver = _version(window)

    def _edits(self, window, stream):
        """Tell the handle what the caller wrote since the last call: the state blob
        (e.g. `env.value[:] = ...`) -> pmenv_state_written; the in-place window (an edit,
        or a different tensor, possibly at the same address) -> pmenv_window_written."""
        sv = _version(self._state)
        if sv is None or sv != self._state_ver:
            _abi.check(self._lib.pmenv_state_written(self._h, stream), self._h, "pmenv_state_written")
            self._state_ver = sv
        elif window is not None and (self._win is None or self._win() is not window or
                                     self._win_ver is None or _version(window) != self._win_ver):
            _abi.check(self._lib.pmenv_window_written(self._h, _ptr(window), stream), self._h,
                       "pmenv_window_written")

    def window_written(self, features):
        """Announce that `features` — the window the next fused step advances in place — was
        written in a way torch's version counter does not see: through `.data`, DLPack /
        CuPy, a raw kernel on `data_ptr()`, or between replays of a captured hipGraph (the
        wrapper's own check runs once, at capture). The next flat step re-reads its tile
        halo from the window (pmenv_window_written)."""
        self._obs_check(features)
        if features.device.type == "cpu":
            return
        _abi.check(self._lib.pmenv_window_written(self._h, _ptr(features), self._stream()), self._h,
                   "pmenv_window_written")
        self._watch(features)

    def state_written(self):
        """Announce a write of the env state (value, ring, counters, statistics) that
        bypassed torch's version counter (see window_written); the next flat step
        re-reads its snapshot from the canonical state (pmenv_state_written)."""
        _abi.check(self._lib.pmenv_state_written(self._h, self._stream()), self._h, "pmenv_state_written")
        self._state_ver = _version(self._state)

    def advance(self, action, features, bar, prices=None, out=None):
        """Fused step: window advance + bar append (see step)."""
        return self.step(action, features, prices=prices, bar=bar, out=out)

    # ------------------------------------------------------------------ state
    def state_dict(self):
        """Checkpoint (value, reward statistics, counters, ring) as one tensor."""
        return {"state": self._state.clone(), "cfg": self.cfg.as_dict()}

    def load_state_dict(self, sd):
        st = sd["state"]
        if st.dtype != torch.uint8 or st.numel() != self._state.numel():
            raise ValueError("state blob mismatch (a uint8 blob of this env shape's size expected)")
        # through pmenv_set_state: the handle re-primes what it derives from the state
        src = st.to(device=self.device, dtype=torch.uint8).contiguous()
        self._hval = None
        _abi.check(self._lib.pmenv_set_state(self._h, _ptr(src), self._stream()), self._h, "pmenv_set_state")

    @property
    def step_path(self):
        """Kernels the fused advance launches for this shape (diagnostics)."""
        return self._lib.pmenv_step_path(self._h).decode()

    def nonfinite_count(self):
        return int(self._nonfinite.item())

    def close(self):
        if getattr(self, "_h", None):
            torch.cuda.synchronize(self.device)
            self._lib.pmenv_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                self._lib.pmenv_destroy(self._h)
                self._h = None
        except Exception:
            pass
