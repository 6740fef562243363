"""An on-policy training loop over B lockstep envs — the shape of train/on_policy.py
(`Train._rollout` :59-67 and `Train._update` :69-74) with the env step, the rollout
storage, the return pass and the trainer reward all on device.

    reference (one env)                         here (B envs, one launch per step each)
    s = env.reset(data)                 :62     env.reset(buf.obs(0))
    a = agent.act(s)                    :64     a = policy(buf.obs(t-1))            (torch, no grad)
    r, s_ = env.step(a, data, prices)   :65     env.step(a, buf.obs(t-1), bar=..., out=buf.obs(t))
    buffer.add(s, a, env.value, r)      :66     buf.add(a, env.value, r)
    for ... in buffer.sample_random():  :71     for s, a, r, _v, _a, p in buf.sample_random(bs):
        agent.update(i, s, a, r, _v, _a, p)         loss = a2c_loss(policy(s), _v, _a, p); step

The policy is any torch module mapping [S, N, W, F] windows to [S, N, 1] scores
(the reference's LSRE-CANN is out of scope; `WindowPolicy` below is a small stand-in).
"""
import torch

from .rollout_buffer import DeviceRolloutBuffer
from .trainer import a2c_loss


class WindowPolicy(torch.nn.Module):
    """Per-asset MLP over the log-price window (a stand-in for net/lsre_cann.py):
    [S, N, W, F] -> [S, N, 1] scores; the batched reward normalises them."""

    def __init__(self, window, features=5, hidden=32):
        super().__init__()
        self.net = torch.nn.Sequential(torch.nn.Linear(window * features, hidden), torch.nn.Tanh(),
                                       torch.nn.Linear(hidden, 1))

    def forward(self, s):
        S, N, W, F = s.shape
        x = s.clone()
        last = x[..., W - 1:W, :F - 1].clamp(min=1e-12)
        x[..., :F - 1] = torch.log(x[..., :F - 1].clamp(min=1e-12) / last)   # prices relative to the last close
        return self.net(x.reshape(S, N, W * F))


class WindowCritic(torch.nn.Module):
    """Value head over the whole window (a stand-in critic: the reference's A2C has
    none): [S, N, W, F] -> [S]."""

    def __init__(self, window, features=5, hidden=32):
        super().__init__()
        self.body = WindowPolicy(window, features, hidden)

    def forward(self, s):
        return self.body(s).mean(dim=(1, 2))


class OnPolicy:
    def __init__(self, env, policy, horizon, series=None, lr=1e-3, batch_size=256, generator=None):
        """series: a pmenv.MarketSeries — every env trades it from its own start day, in
        place, and the rollout buffer keeps actions, w', values and rewards only (compact,
        windows re-materialised at sample time); None: bars fed per step, the env advancing
        straight into the buffer's window slab."""
        cfg = env.cfg
        self.env, self.policy = env, policy
        self.buf = DeviceRolloutBuffer(cfg.num_envs, cfg.num_assets, cfg.window, horizon, cfg.features,
                                       device=env.device, init_cash=cfg.init_cash, close_channel=cfg.close_channel,
                                       series=series, ring=cfg.ring)
        self.optim = torch.optim.Adam(policy.parameters(), lr=lr)
        self.batch_size = batch_size
        self.generator = generator
        self.series = series

    def act(self, s):
        """agent.act (pg.py:29-38): the policy's scores, softmaxed over assets."""
        with torch.no_grad():
            return torch.softmax(self.policy(s).squeeze(-1), dim=-1)

    def rollout(self, obs0=None, bars=None, start=None):
        """train/on_policy.py:59-67 for every env at once. Slab form: obs0 [B, N, W, F] is
        the reset window and bars[t] the day's [B, N, F-1] bars (t = 0 .. horizon-1).
        Compact form (series given at construction): start [B] is every env's first day
        on the series; the window lives in the env (stepped in place) and only the
        action, w', value and reward of each step are recorded."""
        buf, env = self.buf, self.env
        rewards = []
        if buf.compact:
            series = buf.series
            start = torch.as_tensor(start, device=env.device).to(torch.int32).reshape(buf.B)
            buf.reset(start=start)
            obs = series.initial_window(start, buf.W)
            env.reset(obs)
            w = torch.empty(buf.B, buf.N, device=env.device)
            for t in range(1, buf.T + 1):
                a = self.act(obs)
                r, _ = env.step(a, obs, series=series, day=start + buf.W + t - 1, weights_out=w)
                buf.add(a, env.value, r, weights=w)
                rewards.append(r)
            self.obs = obs
            return torch.stack(rewards)
        buf.reset(obs0)
        env.reset(buf.obs(0))
        for t in range(1, buf.T + 1):
            a = self.act(buf.obs(t - 1))
            r, _ = env.step(a, buf.obs(t - 1), bar=bars[t - 1], out=buf.obs(t))
            buf.add(a, env.value, r)
            rewards.append(r)
        return torch.stack(rewards)

    def update(self):
        """train/on_policy.py:69-74 with A2C._loss (a2c.py:40-82) as the fused HIP op."""
        losses = []
        for s, a, r, v_prev, a_prev, p in self.buf.sample_random(self.batch_size, self.generator):
            self.optim.zero_grad(set_to_none=True)
            loss = a2c_loss(self.policy(s), v_prev, a_prev, p)
            loss.backward()
            self.optim.step()
            losses.append(loss.detach())
        return torch.stack(losses) if losses else torch.empty(0)

    def advantages(self, critic, gamma=0.99, lam=0.95, group=None, eps=1e-8):
        """The return pass the north star adds to replay/rollout_buffer.py (which stores
        (s, a, v, r) and computes nothing, :43-57): the critic's values of every stored
        window -> GAE(gamma, lambda) as the HIP scan (DeviceRolloutBuffer.returns) ->
        advantages normalised with moments summed over every rank (pmenv.parallel.normalize:
        HIP moments kernel + one 24-byte all-reduce, RCCL over xGMI under "nccl").
        critic: [S, N, W, F] windows -> [S] (or [S, 1]) values. Returns (normalised
        advantages [T, B], returns [T, B], values [T+1, B])."""
        from . import parallel
        T = len(self.buf)
        with torch.no_grad():
            values = torch.stack([critic(self.buf.obs(t)).reshape(-1) for t in range(T + 1)]).float()
        adv, ret = self.buf.returns(values, gamma, lam)
        return parallel.normalize(adv, group=group, eps=eps), ret, values

    def update_critic(self, critic, optim, returns, batch_size=None, generator=None):
        """Regress the critic on the GAE returns (the value baseline of an actor-critic),
        over random minibatches of the stored (step, env) windows. Returns the losses."""
        T, B = returns.shape
        n = T * B
        bs = n if not batch_size or batch_size < 0 else batch_size
        perm = torch.randperm(n, generator=generator).to(returns.device)
        losses = []
        for i in range(0, n - bs + 1, bs):
            idx = perm[i:i + bs]
            t, env = idx // B, idx % B
            pred = critic(self.buf.windows(t, env)).reshape(-1)
            loss = torch.nn.functional.mse_loss(pred, returns[t, env])
            optim.zero_grad(set_to_none=True)
            loss.backward()
            optim.step()
            losses.append(loss.detach())
        return torch.stack(losses) if losses else torch.empty(0)
