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
    def __init__(self, env, policy, horizon, series=None, lr=1e-3, batch_size=256, generator=None,
                 explore_std=0.0, explore_seed=44, env_offset=0):
        """series: a pmenv.MarketSeries — every env trades it from its own start day, in
        place, and the rollout buffer keeps actions, w', values and rewards only (compact,
        windows re-materialised at sample time); None: bars fed per step, the env advancing
        straight into the buffer's window slab.
        explore_std > 0: the rollout's actions are softmax(scores + explore_std * eps), eps a
        centred N(0, I) draw keyed by (explore_seed, step, global env id, asset) — the
        stochastic policy update_actor_critic scores; env_offset is this rank's first global
        env id (pmenv.parallel.shard_range), so a sharded rollout draws exactly its slice of
        the unsharded one's noise."""
        cfg = env.cfg
        self.env, self.policy = env, policy
        self.buf = DeviceRolloutBuffer(cfg.num_envs, cfg.num_assets, cfg.window, horizon, cfg.features,
                                       device=env.device, init_cash=cfg.init_cash, close_channel=cfg.close_channel,
                                       series=series, ring=cfg.ring)
        self.optim = torch.optim.Adam(policy.parameters(), lr=lr)
        self.batch_size = batch_size
        self.generator = generator
        self.series = series
        self.explore_std = float(explore_std)
        self.explore_seed = int(explore_seed)
        self.env_offset = int(env_offset)
        self._u = None                 # [T, B, N] centred logits the last exploring rollout sampled

    def act(self, s, t=None):
        """agent.act (pg.py:29-38): the policy's scores, softmaxed over assets; with
        exploration, the scores plus the step's centred Gaussian noise (`t`: the rollout step)."""
        with torch.no_grad():
            dtype = next(self.policy.parameters()).dtype
            mu = self.policy(s.to(dtype)).squeeze(-1).float()
            if self.explore_std > 0.0 and t is not None:
                mu = mu + self.explore_std * self._noise[t - 1]
                # the sampled centred logits, scored later by log_prob: recovering them from
                # the softmax action loses them where the softmax underflows
                self._u[t - 1] = mu - mu.mean(dim=-1, keepdim=True)
            return torch.softmax(mu, dim=-1)

    def _draw_noise(self):
        """[T, B, N] centred N(0, I) logits: the log of a synth.actions draw (a softmax of
        N(0, 1) logits keyed by step, global env id and asset) minus its mean over assets."""
        from . import synth
        buf = self.buf
        la = torch.log(synth.actions(buf.T, buf.B, buf.N, env_offset=self.env_offset, seed=self.explore_seed,
                                     device=self.env.device))
        self._noise = la - la.mean(dim=-1, keepdim=True)
        self._u = torch.empty_like(self._noise)          # [T, B, N] sampled centred logits (act)

    def rollout(self, obs0=None, bars=None, start=None):
        """train/on_policy.py:59-67 for every env at once. Slab form: obs0 [B, N, W, F] is
        the reset window and bars[t] the day's [B, N, F-1] bars (t = 0 .. horizon-1).
        Compact form (series given at construction): start [B] is every env's first day
        on the series; the window lives in the env (stepped in place) and only the
        action, w', value and reward of each step are recorded."""
        buf, env = self.buf, self.env
        rewards = []
        if self.explore_std > 0.0:
            self._draw_noise()
        if buf.compact:
            series = buf.series
            start = torch.as_tensor(start, device=env.device).to(torch.int32).reshape(buf.B)
            buf.reset(start=start)
            obs = series.initial_window(start, buf.W)
            env.reset(obs)
            w = torch.empty(buf.B, buf.N, device=env.device)
            for t in range(1, buf.T + 1):
                a = self.act(obs, t)
                r, _ = env.step(a, obs, series=series, day=start + buf.W + t - 1, weights_out=w)
                buf.add(a, env.value, r, weights=w)
                rewards.append(r)
            self.obs = obs
            return torch.stack(rewards)
        buf.reset(obs0)
        env.reset(buf.obs(0))
        for t in range(1, buf.T + 1):
            a = self.act(buf.obs(t - 1), t)
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
        dtype = next(critic.parameters()).dtype
        with torch.no_grad():
            values = torch.stack([critic(self.buf.obs(t).to(dtype)).reshape(-1) for t in range(T + 1)]).float()
        adv, ret = self.buf.returns(values, gamma, lam)
        return parallel.normalize(adv, group=group, eps=eps), ret, values

    def log_prob(self, s, a, u=None):
        """log pi(a | s) of the exploring policy, up to a constant: the action's centred
        logits u against the centred scores mu under N(mu, explore_std^2) on the simplex's
        logit plane (softmax is shift-invariant, so only centred logits matter).
        s [S, N, W, F], a [S, N] -> [S]. u [S, N]: the centred logits act() sampled (exact);
        None recovers them as the centred log of a, which is biased where the softmax
        underflowed (a warning names how many actions hold such weights)."""
        mu = self.policy(s).squeeze(-1)
        mu = mu - mu.mean(dim=-1, keepdim=True)
        if u is None:
            tiny = torch.finfo(torch.float32).tiny
            if bool((a < 1e-30).any()):
                import warnings
                warnings.warn(f"log_prob: {int((a < 1e-30).any(dim=-1).sum())} actions hold softmax weights "
                              "below 1e-30; their logits are not recoverable from the action (pass u)")
            la = torch.log(a.to(mu.dtype).clamp(min=tiny))
            u = la - la.mean(dim=-1, keepdim=True)
        return -((u.to(mu.dtype) - mu) ** 2).sum(dim=-1) / (2.0 * self.explore_std ** 2)

    def update_actor_critic(self, adv, group=None, chunk=None):
        """One actor-critic policy step on the normalised advantages advantages() returns
        ([T, B], the output of the 24-byte moment all-reduce): the loss
        -sum(adv[t-1, b] * log pi(a_t | s_{t-1})) / n over every stored (step, env) pair,
        n the pairs of all ranks. The gradient is accumulated over `chunk` pairs at a time
        (None: all at once), then the per-rank gradient sums, the loss sum and the pair
        count go through ONE all-reduce (pmenv.parallel.allreduce_grads: RCCL under "nccl")
        and every rank takes the same optimizer step — so the sharded update equals the
        unsharded one up to floating-point reassociation. Returns the global loss.
        The reference's A2C has no critic (a2c.py:40-82); this is the consumer of the
        north star's advantage-normalisation moments. Needs explore_std > 0."""
        from . import parallel
        if self.explore_std <= 0.0:
            raise ValueError("update_actor_critic scores a stochastic policy: construct OnPolicy with explore_std > 0")
        buf = self.buf
        T, B = adv.shape
        if T != len(buf) or B != buf.B:
            raise ValueError(f"advantages must be [{len(buf)}, {buf.B}]")
        n = T * B
        cs = n if not chunk or chunk < 0 else int(chunk)
        self.optim.zero_grad(set_to_none=True)
        loss_sum = torch.zeros((), dtype=torch.float64, device=adv.device)
        dtype = next(self.policy.parameters()).dtype
        for i in range(0, n, cs):
            idx = torch.arange(i, min(i + cs, n), device=adv.device)
            t, env = idx // B + 1, idx % B
            s, a, _r, _v, _a, _p = buf.gather(t, env)
            u = None if self._u is None else self._u[t - 1, env]      # None: a buffer filled without act()
            lp = self.log_prob(s.to(dtype), a.reshape(-1, buf.N), u=u)
            loss = -(adv[t - 1, env].to(dtype) * lp).sum()
            loss.backward()
            loss_sum += loss.detach().double()
        total, count = parallel.allreduce_grads(list(self.policy.parameters()), loss_sum, float(n), group=group)
        self.optim.step()
        return total / count

    def update_critic(self, critic, optim, returns, batch_size=None, generator=None, group=None):
        """Regress the critic on the GAE returns (the value baseline of an actor-critic),
        over random minibatches of the stored (step, env) windows. group: the ranks'
        gradients are averaged (one all-reduce per minibatch) so replicated critics stay
        equal. Returns the losses."""
        from . import parallel
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
            if group is not None or parallel.world() > 1:
                parallel.allreduce_grads(list(critic.parameters()), loss.detach().double(), 1.0, group=group)
            optim.step()
            losses.append(loss.detach())
        return torch.stack(losses) if losses else torch.empty(0)
