"""Device rollout storage for B lockstep envs (the on-policy caller of the env step).

Mirrors replay/rollout_buffer.py (`RolloutBuffer` :7-142) with a leading env
dimension, resident in HBM:

    reference                                   here
    RolloutBuffer(feat, train_len, prices) :8   DeviceRolloutBuffer(num_envs, num_assets, window, horizon)
    reset()                            :29-41   reset(obs0)     row 0 = a e0 / v INITIAL_CASH / r 0 (:36-39)
    add(s, a, v, r)                    :43-57   add(a, v, r)    s is not copied: see below
    sample()                           :59-101  sample(batch_size)         in-order minibatches
    sample_random()                    :103-142 sample_random(batch_size)  random minibatches
      -> (s, a, r, _v, _a, p)                     the same six tensors, the same shapes

Two storage forms for the observations s:

* compact (series=MarketSeries; SURVEY.md §8f f1 — the device rollout keeps actions,
  rewards and values only): the envs step their own windows in place on the resident
  series, and the buffer keeps per step the action, the env's post-drift weights w'
  (info["actions"], trading_env.py:83-85), the value and the reward — O(T·B·N). The
  windows are re-materialised at sample time by pmenv_rollout_gather from the series
  (market channels) and the w' history (the weight channel, in the ring order
  weight_buffer.py:32-44 returns). 65,536 envs x 64 steps x 30 assets: ~1 GB.
* slab (bars fed per step): the env advances its window straight into the buffer's
  next slot (double-buffered step, `out=`), so slot t holds the observation after t
  steps at zero extra traffic; [T+1, B, N, W, F] (64 steps of 65,536 envs x 30 x 50 x 5
  = 126 GB of a 288 GB MI355X) — for bar feeds that are not a resident series.

The price relatives p are not stored in either form: p[t] = close_t / close_{t-1} of
the window's last day, the same fp32 quotient the env formed (instrument.py:79).

`returns(values, gamma, lam)` runs the GAE / discounted-return pass over the stored
rewards on device (pmenv_gae_ex).
"""
import ctypes

import torch

from . import _abi, rollout


class DeviceRolloutBuffer:
    def __init__(self, num_envs, num_assets, window, horizon, features=5, device=None, init_cash=25000.0,
                 close_channel=3, series=None, ring="storage"):
        self.B, self.N, self.W, self.F, self.T = num_envs, num_assets, window, features, horizon
        self.device = torch.device(device or (series.device if series is not None else "cuda"))
        self.init_cash = float(init_cash)
        self.close_ch = close_channel
        self.series = series
        self.ring = ring
        if series is not None:
            if series.num_assets != num_assets or series.channels != features - 1:
                raise ValueError("series must be [T, num_assets, features - 1]")
            self.s = None
            self.start = torch.zeros(num_envs, dtype=torch.int32, device=self.device)
            self.w = torch.zeros(horizon, num_envs, num_assets, device=self.device)    # w' of updates 1..T
        else:
            self.s = torch.empty(horizon + 1, num_envs, num_assets, window, features, device=self.device)
        self.a = torch.zeros(horizon + 1, num_envs, num_assets, device=self.device)
        self.v = torch.zeros(horizon + 1, num_envs, dtype=torch.float64, device=self.device)
        self.r = torch.zeros(horizon + 1, num_envs, device=self.device)
        self.step = 1

    @property
    def compact(self):
        return self.s is None

    def nbytes(self):
        """Device bytes held by the buffer."""
        ts = [self.a, self.v, self.r] + ([self.start, self.w] if self.compact else [self.s])
        return sum(t.numel() * t.element_size() for t in ts)

    # ---------------------------------------------------------------- filling
    def reset(self, obs0=None, start=None):
        """rollout_buffer.py:29-41: row 0 is the reset state (a = e0, cash only;
        v = INITIAL_CASH; r = 0). Slab: obs0 (the reset window) goes to slot 0 unless the
        env was reset into slot 0 directly (obs(0)). Compact: start [B] is the first day
        of every env's reset window on the series."""
        if self.compact:
            if start is None:
                raise ValueError("the compact buffer needs the envs' start days")
            self.start.copy_(torch.as_tensor(start).reshape(self.B))
            self.w.zero_()
        elif obs0 is not None and obs0.data_ptr() != self.s[0].data_ptr():
            self.s[0].copy_(obs0)
        self.a.zero_()
        self.a[0, :, 0] = 1.0
        self.v.zero_()
        self.v[0] = self.init_cash
        self.r.zero_()
        self.step = 1

    def obs(self, t):
        """Window after t steps, [B, N, W, F]: a view of the slab (pass it as `features` /
        `out`), or — compact — a fresh tensor re-materialised from the series."""
        if not self.compact:
            return self.s[t]
        env = torch.arange(self.B, dtype=torch.int32, device=self.device)
        return self.windows(torch.full((self.B,), t, dtype=torch.int32, device=self.device), env)

    def add(self, a, v, r, weights=None):
        """rollout_buffer.py:43-57 for every env: the action of this step, the env's
        value after it and its reward (compact: and the post-drift weights w' the step
        produced). The slab's window is already in obs(step)."""
        t = self.step
        if t > self.T:
            raise IndexError(f"rollout buffer full ({self.T} steps)")
        if self.compact:
            if weights is None:
                raise ValueError("the compact buffer records the step's post-drift weights")
            self.w[t - 1].copy_(weights.reshape(self.B, self.N))
        self.a[t].copy_(a.reshape(self.B, self.N))
        self.v[t].copy_(v.reshape(self.B))
        self.r[t].copy_(r.reshape(self.B))
        self.step = t + 1

    def __len__(self):
        return self.step - 1

    # ---------------------------------------------------------------- reading
    def windows(self, t, env):
        """Windows after t[j] steps of envs env[j], [S, N, W, F]."""
        t = t.to(self.device, torch.int32).contiguous()
        env = env.to(self.device, torch.int32).contiguous()
        if not self.compact:
            return self.s[t.long(), env.long()]
        S = t.numel()
        out = torch.empty(S, self.N, self.W, self.F, device=self.device)
        lib = _abi.load()
        sb = self.series.bars
        p = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
        st = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        ring = _abi.RING_MODES[self.ring]
        _abi.check(lib.pmenv_rollout_gather(p(sb), sb.shape[0], self.N, self.F, self.W, p(self.start), p(self.w),
                                            self.T, self.B, ring, p(t), p(env), S, p(out), st),
                   None, "pmenv_rollout_gather")
        return out

    def _close(self, t, env):
        """close of the last day of the windows after t steps, [S, N]."""
        if not self.compact:
            return self.s[t, env, :, self.W - 1, self.close_ch]
        day = self.start[env].long() + t + self.W - 1
        return self.series.bars[day, :, self.close_ch]

    def price_relatives(self, t):
        """p of step t (1 <= t < step): close_t / close_{t-1} of every asset, [B, N]."""
        env = torch.arange(self.B, device=self.device)
        tt = torch.full((self.B,), t, dtype=torch.long, device=self.device)
        return self._close(tt, env) / self._close(tt - 1, env)

    def gather(self, t, env):
        """(s, a, r, _v, _a, p) of the (step, env) pairs, shaped like the reference's
        batches: s [S, N, W, F] (the window the action was taken on), a / _a / p
        [S, N, 1], r / _v [S, 1, 1]."""
        t = t.to(self.device, torch.long)
        env = env.to(self.device, torch.long)
        S = t.numel()
        s = self.windows(t - 1, env)                                  # rollout_buffer.py:128
        a = self.a[t, env].reshape(S, self.N, 1)                      # :129
        r = self.r[t, env].reshape(S, 1, 1)                           # :130
        v_prev = self.v[t - 1, env].to(torch.float32).reshape(S, 1, 1)   # :131
        a_prev = self.a[t - 1, env].reshape(S, self.N, 1)             # :132
        # :133 — only the last day's close of the next window is read (no [S, N, W, F]
        # copy of the next windows)
        p = (self._close(t, env) / s[..., self.W - 1, self.close_ch]).reshape(S, self.N, 1)
        return s, a, r, v_prev, a_prev, p

    def _pairs(self, order):
        """flat index -> (step 1.., env): step-major, like the reference's [epoch_len] axis."""
        return order // self.B + 1, order % self.B

    def sample(self, batch_size):
        """rollout_buffer.py:59-101: consecutive minibatches over (step, env), step-major."""
        n = len(self) * self.B
        bs = n if batch_size == -1 else batch_size
        for i in range(0, n - bs + 1, bs):
            yield self.gather(*self._pairs(torch.arange(i, i + bs, device=self.device)))

    def sample_random(self, batch_size, generator=None):
        """rollout_buffer.py:103-142: random minibatches without replacement."""
        n = len(self) * self.B
        bs = n if batch_size == -1 else batch_size
        perm = torch.randperm(n, generator=generator).to(self.device)
        for i in range(0, n - bs + 1, bs):
            yield self.gather(*self._pairs(perm[i:i + bs]))

    def returns(self, values, gamma=0.99, lam=0.95, dones=None):
        """GAE over the stored rollout: values [T+1, B] (critic, bootstrap row last),
        rewards r[1..T]. Returns (advantages, returns), [T, B] float32."""
        T = len(self)
        return rollout.gae(self.r[1:T + 1], values, dones, gamma, lam)
