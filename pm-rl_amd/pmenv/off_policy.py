"""An off-policy training loop over B lockstep envs — the shape of train/off_policy.py
(`Train._collect_rand` :60-71, `_collect` :73-86, `_update_off_policy` :88-94,
`_evaluate_off_policy` :96-110) with the market data, the env step, the replay buffer
and the evaluation metrics all on device.

    reference (one env)                          here (B envs)
    self.s = env.reset(feat)             :65     obs = series.initial_window(start, W); env.reset(obs)
    a = agent.act(s, is_random=True)     :67     a = random simplex weights           (collect_rand)
    a = agent.act(s)                     :81     a = act(obs)                          (torch, no grad)
    r, s_ = env.step(a, feat, targ)      :68     env.step(a, obs, series=series, day=day)   in place
    buffer.add(epoch, step, a, r)        :69     replay.add(day - 1, a, r)             (DeviceReplay)
    s, a, r, s_ = buffer.sample()        :91     replay.sample(batch_size)             (HIP gather)
    agent.update(epoch, step, s, a, r, s_) :92   update(s, a, r, s_)                   (caller's agent)
    metrics.write()                      :110    trajectory_metrics(...)               (HIP reductions)

Every env trades the one HBM-resident series (pmenv.data.MarketSeries) from its own
start day: the step reads day[b]'s bar straight from the series (no per-step host
feed). The agent (DSAC / TD3 / DreamerV3 in the reference) is out of scope: `act`
and `update` are the caller's callables.
"""
import torch

from .replay import DeviceReplay, trajectory_metrics


class OffPolicy:
    def __init__(self, env, series, capacity, act=None, update=None, batch_size=256, generator=None):
        """env: a pmenv.TradingEnv over B envs; series: pmenv.data.MarketSeries [T, N, F-1];
        capacity: replay steps kept per env (buffer.py's ring); act(obs [B, N, W, F]) ->
        [B, N] weights; update(s, a, r, s_) -> anything (one agent update)."""
        cfg = env.cfg
        if series.num_assets != cfg.num_assets or series.channels != cfg.features - 1:
            raise ValueError("series must be [T, num_assets, features - 1]")
        self.env, self.series = env, series
        self.B, self.N, self.W = cfg.num_envs, cfg.num_assets, cfg.window
        self.replay = DeviceReplay(self.B, self.N, self.W, capacity, series, cfg.features)
        self.act_fn, self.update_fn = act, update
        self.batch_size = batch_size
        self.generator = generator

    def _random_action(self):
        """agent.act(s, is_random=True): uniform random portfolio weights (a simplex point)."""
        g = torch.empty(self.B, self.N, device=self.env.device).exponential_()
        return g / g.sum(-1, keepdim=True)

    def collect(self, start, steps, random=False):
        """_collect_rand / _collect (off_policy.py:60-86) for every env: reset on the window
        ending the day before start + W, then `steps` steps, each recorded in the replay.
        start: [B] first day of each env's initial window. Returns (rewards [steps, B], obs)."""
        start = torch.as_tensor(start, device=self.env.device).to(torch.int32).reshape(self.B)
        if int(start.max()) + self.W + steps > self.series.days:
            raise ValueError("series too short for start + window + steps")
        obs = self.series.initial_window(start, self.W)
        self.env.reset(obs)
        self.replay.new_episode()                 # no sampled window spans the reset
        day = start + self.W                      # the bar each env appends next
        rewards = []
        for _ in range(steps):
            if random or self.act_fn is None:
                a = self._random_action()
            else:
                with torch.no_grad():
                    a = self.act_fn(obs)
            r, _ = self.env.step(a, obs, series=self.series, day=day)
            self.replay.add(day - 1, a, r)        # the day of the window the action was taken on
            rewards.append(r)
            day = day + 1
        return torch.stack(rewards), obs

    def update(self, steps):
        """_update_off_policy (off_policy.py:88-94): `steps` sampled batches into update()."""
        out = []
        for _ in range(steps):
            s, a, r, s_ = self.replay.sample(self.batch_size, self.generator)
            out.append(self.update_fn(s, a, r, s_) if self.update_fn is not None else None)
        return out

    def evaluate(self, start, steps, act=None):
        """_evaluate_off_policy (off_policy.py:96-110) + Metrics (util/eval.py:14-37): a
        deterministic run of `steps` days from `start`, then per-env Sharpe, Sortino,
        max drawdown, average turnover and final value ({name: [B] f64})."""
        act = act or self.act_fn
        env = self.env
        track = env.track_info
        env.track_info = True
        try:
            start = torch.as_tensor(start, device=env.device).to(torch.int32).reshape(self.B)
            obs = self.series.initial_window(start, self.W)
            env.reset(obs)
            day = start + self.W
            for _ in range(steps):
                with torch.no_grad():
                    a = act(obs) if act is not None else self._random_action()
                env.step(a, obs, series=self.series, day=day)
                day = day + 1
            rets = torch.stack(env.info["returns"][1:]) - 1.0          # [T, B] simple returns
            vals = torch.stack(env.info["values"])                     # [T+1, B]
            wts = torch.stack(env.info["actions"])                     # [T+1, B, N] post-drift weights
            return trajectory_metrics(rets, vals, wts)
        finally:
            env.track_info = track
