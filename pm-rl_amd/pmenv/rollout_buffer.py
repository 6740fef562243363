"""Device rollout storage for B lockstep envs (the on-policy caller of the env step).

Mirrors replay/rollout_buffer.py (`RolloutBuffer` :7-142) with a leading env
dimension, resident in HBM:

    reference                                   here
    RolloutBuffer(feat, train_len, prices) :8   DeviceRolloutBuffer(num_envs, num_assets, window, horizon)
    reset()                            :29-41   reset(obs0)     row 0 = a e0 / v INITIAL_CASH / r 0 (:36-39)
    add(s, a, v, r)                    :43-57   add(a, v, r)    s is already stored: see below
    sample()                           :59-101  sample(batch_size)         in-order minibatches
    sample_random()                    :103-142 sample_random(batch_size)  random minibatches
      -> (s, a, r, _v, _a, p)                     the same six tensors, the same shapes

The windows are not copied into the buffer: the env advances its window straight
into the buffer's next slot (double-buffered step, `out=`), so slot t holds the
observation after t steps — the reference's s[t+1] — at zero extra traffic, and the
[T+1, B, N, W, F] slab is the rollout (HBM-sized: 64 steps of 65,536 envs x 30
assets x 50 days = 126 GB of a 288 GB MI355X). The price relatives p are not stored
either: p[t] = close(window t)[W-1] / close(window t-1)[W-1], the same fp32 quotient
the env formed (instrument.py:79).

`returns(values, gamma, lam)` runs the GAE / discounted-return pass over the stored
rewards on device (pmenv_gae_ex).
"""
import torch

from . import rollout


class DeviceRolloutBuffer:
    def __init__(self, num_envs, num_assets, window, horizon, features=5, device=None, init_cash=25000.0,
                 close_channel=3):
        self.B, self.N, self.W, self.F, self.T = num_envs, num_assets, window, features, horizon
        self.device = torch.device(device or "cuda")
        self.init_cash = float(init_cash)
        self.close_ch = close_channel
        self.s = torch.empty(horizon + 1, num_envs, num_assets, window, features, device=self.device)
        self.a = torch.zeros(horizon + 1, num_envs, num_assets, device=self.device)
        self.v = torch.zeros(horizon + 1, num_envs, dtype=torch.float64, device=self.device)
        self.r = torch.zeros(horizon + 1, num_envs, device=self.device)
        self.step = 1

    # ---------------------------------------------------------------- filling
    def reset(self, obs0=None):
        """rollout_buffer.py:29-41: row 0 is the reset state (a = e0, cash only;
        v = INITIAL_CASH; r = 0). obs0 (the reset window) goes to slot 0 unless the
        env was reset into slot 0 directly (obs(0))."""
        if obs0 is not None and obs0.data_ptr() != self.s[0].data_ptr():
            self.s[0].copy_(obs0)
        self.a.zero_()
        self.a[0, :, 0] = 1.0
        self.v.zero_()
        self.v[0] = self.init_cash
        self.r.zero_()
        self.step = 1

    def obs(self, t):
        """Window after t steps, [B, N, W, F] (a view: pass it as `features` / `out`)."""
        return self.s[t]

    def add(self, a, v, r):
        """rollout_buffer.py:43-57 for every env: the action of this step, the env's
        value after it and its reward. The step's window is already in obs(step)."""
        t = self.step
        if t > self.T:
            raise IndexError(f"rollout buffer full ({self.T} steps)")
        self.a[t].copy_(a.reshape(self.B, self.N))
        self.v[t].copy_(v.reshape(self.B))
        self.r[t].copy_(r.reshape(self.B))
        self.step = t + 1

    def __len__(self):
        return self.step - 1

    # ---------------------------------------------------------------- reading
    def price_relatives(self, t):
        """p of step t (1 <= t < step): close_t / close_{t-1} of every asset, [B, N]."""
        c = self.close_ch
        return self.s[t][..., self.W - 1, c] / self.s[t - 1][..., self.W - 1, c]

    def gather(self, t, env):
        """(s, a, r, _v, _a, p) of the (step, env) pairs, shaped like the reference's
        batches: s [S, N, W, F] (the window the action was taken on), a / _a / p
        [S, N, 1], r / _v [S, 1, 1]."""
        t = t.to(self.device, torch.long)
        env = env.to(self.device, torch.long)
        S = t.numel()
        c = self.close_ch
        s = self.s[t - 1, env]                                        # rollout_buffer.py:128
        a = self.a[t, env].reshape(S, self.N, 1)                      # :129
        r = self.r[t, env].reshape(S, 1, 1)                           # :130
        v_prev = self.v[t - 1, env].to(torch.float32).reshape(S, 1, 1)   # :131
        a_prev = self.a[t - 1, env].reshape(S, self.N, 1)             # :132
        # :133 — only the last day's close of the next window is read (indexing the slab
        # directly: no [S, N, W, F] copy of the next windows)
        p = (self.s[t, env, :, self.W - 1, c] / s[..., self.W - 1, c]).reshape(S, self.N, 1)
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
