"""Device replay for vectorised envs.

`DeviceReplay` mirrors replay/buffer.py (`ReplayBuffer.add` :23-37, `.sample` :39-79):
per recorded step it keeps only the day index of the window the agent acted on,
the action and the reward; `sample` re-materialises the observation windows s, s'
on device from the resident market series (pmenv.data.MarketSeries) with the last W
actions as the weight channel, exactly as the reference rebuilds them from its
dataset. `trajectory_metrics` restates util/eval.py:14-37 (Sharpe, Sortino, max
drawdown, average turnover) per env on device.
"""
import ctypes

import numpy as np
import torch

from . import _abi
from .config import RISK_FREE_RATE


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def valid_starts(row_episode, oldest, count, W, H):
    """Offsets st (from the oldest recorded row) whose W+1 rows st .. st+W all belong to
    one episode — the reference samples a window inside one epoch of its [epoch, step]
    layout (buffer.py:17-21, :47-51). Episode ids only grow along the ring, so the
    first and the last row of a window decide. st < count - W - 1, as buffer.py:50
    draws starts below epoch_len - WINDOW_SIZE - 1. Returns a range when every start is
    valid (the oldest and the newest row share one episode: no scan), else an int64 array."""
    span = max(count - W - 1, 0)
    ep = np.asarray(row_episode)
    if span == 0 or ep[oldest] == ep[(oldest + count - 1) % H]:
        return range(span)
    chrono = np.roll(ep, -oldest)[:count]                 # rows oldest .. newest
    return np.flatnonzero(chrono[:span] == chrono[W:W + span])


class DeviceReplay:
    def __init__(self, num_envs, num_assets, window, capacity, series, features=5):
        if capacity < window + 2:
            raise ValueError("capacity must hold at least window + 2 steps")
        self.B, self.N, self.W, self.F, self.H = num_envs, num_assets, window, features, capacity
        self.series = series
        dev = series.device
        self.days = torch.zeros(capacity, num_envs, dtype=torch.int32, device=dev)
        self.actions = torch.zeros(capacity, num_envs, num_assets, dtype=torch.float32, device=dev)
        self.rewards = torch.zeros(capacity, num_envs, dtype=torch.float32, device=dev)
        self.head = 0
        self.count = 0
        # episode id of every ring row (all envs record in lockstep, so one id per row)
        self.episode = 0
        self._row_ep = np.zeros(capacity, dtype=np.int64)
        self._starts = None           # device tensor of valid starts when some windows straddle episodes
        self._starts_key = None

    def __len__(self):
        return self.count

    def new_episode(self):
        """Steps added from now on belong to a new episode (the env was reset): no sampled
        window spans the boundary (buffer.py keeps each epoch in its own row)."""
        self.episode += 1

    def add(self, day, action, reward):
        """buffer.py:23-37: one recorded step for every env."""
        h = self.head
        self.days[h].copy_(torch.as_tensor(day).reshape(self.B))
        self.actions[h].copy_(torch.as_tensor(action).reshape(self.B, self.N))
        self.rewards[h].copy_(torch.as_tensor(reward).reshape(self.B))
        self._row_ep[h] = self.episode
        self.head = (h + 1) % self.H
        self.count = min(self.count + 1, self.H)

    def indices(self, batch_size, generator=None):
        """Random (start, env) pairs with W+1 consecutive recorded steps of one episode
        (buffer.py:47-51)."""
        span = self.count - self.W - 1
        if span < 1:
            raise ValueError("not enough recorded steps to sample a window")
        # drawn where the generator lives: a CPU generator (reproducible across devices)
        # costs a host->device copy per batch; no generator or a device one stays on the GPU
        dev = self.days.device
        gdev = generator.device if generator is not None else dev
        oldest = (self.head - self.count) % self.H
        first, last = int(self._row_ep[oldest]), int(self._row_ep[(oldest + self.count - 1) % self.H])
        key = None if first == last else (oldest, self.count, first, last)
        if key is None:                    # one episode in the ring: every start (no scan, no upload)
            self._starts_key, self._starts = None, None
        elif self._starts_key != key:
            self._starts_key = key
            ok = valid_starts(self._row_ep, oldest, self.count, self.W, self.H)
            if len(ok) == 0:
                raise ValueError("no episode holds W + 1 recorded steps")
            self._starts = None if len(ok) == span else torch.as_tensor(ok, dtype=torch.int64).to(gdev)
        if self._starts is None:
            st = torch.randint(0, span, (batch_size,), generator=generator, device=gdev)
        else:
            if self._starts.device != torch.device(gdev):
                self._starts = self._starts.to(gdev)
            st = self._starts[torch.randint(0, self._starts.numel(), (batch_size,), generator=generator, device=gdev)]
        env = torch.randint(0, self.B, (batch_size,), generator=generator, device=gdev)
        h0 = (oldest + st) % self.H
        return h0.to(dev, torch.int32), env.to(dev, torch.int32)

    def gather(self, h0, env):
        """buffer.py:53-79 for the given samples: (s, a, r, s_next) shaped like the reference."""
        lib = _abi.load()
        S = h0.numel()
        dev = self.days.device
        s = torch.empty(S, self.N, self.W, self.F, device=dev)
        s2 = torch.empty_like(s)
        a = torch.empty(S, self.N, device=dev)
        r = torch.empty(S, device=dev)
        sb = self.series.bars
        st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        _abi.check(lib.pmenv_replay_gather(_p(sb), sb.shape[0], self.N, self.F, self.W, _p(self.days),
                                           _p(self.actions), _p(self.rewards), self.H, self.B,
                                           _p(h0.contiguous()), _p(env.contiguous()), S, _p(s), _p(s2), _p(a), _p(r),
                                           st), None, "pmenv_replay_gather")
        return s, a.reshape(S, self.N, 1), r.reshape(S, 1, 1), s2

    def sample(self, batch_size, generator=None):
        return self.gather(*self.indices(batch_size, generator))


def trajectory_metrics(returns, values, weights, risk_free_rate=RISK_FREE_RATE, periods=252):
    """Per-env {sharpe, sortino, max_drawdown, average_turnover, final_value} over a
    trajectory: returns [T, B] simple returns, values [T+1, B], weights [T+1, B, N]."""
    lib = _abi.load()
    r = returns.to(torch.float64).contiguous()
    T, B = r.shape
    v = values.to(device=r.device, dtype=torch.float64).contiguous()
    w = weights.to(device=r.device, dtype=torch.float32).contiguous()
    if tuple(v.shape) != (T + 1, B) or w.shape[:2] != (T + 1, B):
        raise ValueError("values must be [T+1, B] and weights [T+1, B, N]")
    out = torch.empty(B, 5, dtype=torch.float64, device=r.device)
    st = ctypes.c_void_p(torch.cuda.current_stream(r.device).cuda_stream)
    _abi.check(lib.pmenv_metrics(_p(r), _p(v), _p(w), T, B, w.shape[2], float(risk_free_rate), float(periods),
                                 _p(out), st), None, "pmenv_metrics")
    keys = ("sharpe", "sortino", "max_drawdown", "average_turnover", "final_value")
    return {k: out[:, i] for i, k in enumerate(keys)}
