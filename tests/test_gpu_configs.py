"""BASELINE.json configs 2, 3 and 5 at their full sizes on one MI355X, each checked
against the CPU oracle (or an independent env / the numpy restatement), not
against itself. Needs a GPU.

  config 2: 4,096 envs x 30 assets, A2C on-policy (train/on_policy.py:59-74)
  config 3: 16,384 envs x 30 assets, off-policy + device replay (train/off_policy.py,
            replay/buffer.py:39-79)
  config 5: 8,192 envs x 500 assets, differential-Sharpe reward (the asset stress)
"""
import numpy as np
import pytest
import torch

from oracle import OracleEnv

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(DEV)


class _OracleTrack:
    """The first S envs of a FULL-SIZE handle against the CPU oracle on the same inputs,
    step by step (the handle's own geometry, tiles and step path — not a side handle of
    S envs): rewards within |d| <= 1e-6 |r| + 1e-9, values rtol 1e-12, and the windows'
    market channels bit-exact (weight channel rtol 2e-7) whenever a window is checked."""

    def __init__(self, obs0, S, N, W, **cfg_kw):
        from pmenv.config import EnvConfig
        self.S = S
        self.env = OracleEnv(EnvConfig(num_envs=S, num_assets=N, window=W, **cfg_kw))
        self.obs = obs0[:S].cpu().numpy().copy()
        self.env.reset(self.obs)
        self.steps = 0

    def step(self, act, bar, r, value):
        S = self.S
        cr, _, _ = self.env.step(act[:S].cpu().numpy(), self.obs, bar=bar[:S].cpu().numpy())
        g = r[:S].cpu().numpy().astype(np.float64)
        both_nan = np.isnan(g) & np.isnan(cr)
        err = np.where(both_nan, 0.0, np.abs(g - cr))
        assert np.all(err <= 1e-6 * np.abs(np.nan_to_num(cr)) + 1e-9), \
            f"step {self.steps}: reward err {err.max():.3e}"
        np.testing.assert_allclose(value[:S].cpu().numpy(), self.env.value, rtol=1e-12)
        self.steps += 1

    def window(self, obs):
        o = obs[:self.S].cpu().numpy()
        assert np.array_equal(o[..., :4], self.obs[..., :4]), f"market channels after {self.steps} steps"
        np.testing.assert_allclose(o[..., 4], self.obs[..., 4], rtol=2e-7, atol=1e-12)


@pytest.mark.parametrize("commission", [0.0, 0.0025])
def test_gpu_config5_8192x500_diff_sharpe(commission):
    """Config 5 (8,192 envs x 500 assets x 50 days x 5, differential Sharpe) through the
    default in-place path for T = 256 days (five ring wraps): every env's window equals
    the sliding series, the weight channel equals the ring (get_all), values and rewards
    are finite; EVERY env's reward at EVERY step equals a torch f64 restatement of the
    differential Sharpe recursion over the env's own returns (|d| <= 1e-6 |r| + 1e-9; the
    largest fraction of that budget used is printed: DESIGN.md §4 records it); and the
    handle's own first 64 envs match the CPU oracle at every step, with and without
    commission."""
    from pmenv import TradingEnv, synth
    B, N, W, T = 8192, 500, 50, 256
    ser = synth.series(W + T, B, N, seed=51, device=DEV)
    act = synth.actions(T, B, N, seed=52, device=DEV)
    obs = synth.window_from_series(ser, W)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, reward="diff_sharpe",
                     commission=commission, track_info=True)
    track = _OracleTrack(obs, 64, N, W, reward="diff_sharpe", commission=commission)
    env.reset(obs)
    eta = env.cfg.sharpe_eta
    A = torch.zeros(B, dtype=torch.float64, device=DEV)
    Bm = torch.zeros(B, dtype=torch.float64, device=DEV)
    worst_budget, worst_rel = 0.0, 0.0
    for t in range(T):
        r, _ = env.step(act[t], obs, bar=ser[W + t])
        assert bool(torch.isfinite(r).all()) and bool(torch.isfinite(env.value).all())
        ret = env.info["returns"][-1]
        for k in env.info:                                 # keep only the latest record
            del env.info[k][:-1]
        if commission == 0.0:
            y = (ser[W + t, ..., 3] / ser[W + t - 1, ..., 3]).double()
            assert torch.allclose(ret, (act[t].double() * y).sum(-1), rtol=1e-12)
        R = ret - 1.0
        dA, dB, var = R - A, R * R - Bm, Bm - A * A
        ref = torch.where(var > 1e-12, (Bm * dA - 0.5 * A * dB) / (var * var.clamp(min=0).sqrt()),
                          torch.zeros_like(var))
        err = (r.double() - ref).abs()
        budget = err / (1e-6 * ref.abs() + 1e-9)
        assert bool((budget <= 1.0).all()), f"step {t}: {float(err.max()):.3e}"
        worst_budget = max(worst_budget, float(budget.max()))
        big = ref.abs() > 1e-3
        if bool(big.any()):
            worst_rel = max(worst_rel, float((err[big] / ref.abs()[big]).max()))
        A, Bm = A + eta * dA, Bm + eta * dB
        track.step(act[t], ser[W + t], r, env.value)
    print(f"diff-Sharpe, commission {commission}, {T} steps x {B} envs: max |d| / (1e-6 |r| + 1e-9) = "
          f"{worst_budget:.3e}, max |d| / |r| (|r| > 1e-3) = {worst_rel:.3e}")
    assert torch.equal(obs[..., :4], ser[T:T + W].permute(1, 2, 0, 3))
    assert torch.equal(obs[..., 4], env.weights.get_all())
    assert bool(env.weights.is_full.all()) and env.nonfinite_count() == 0
    track.window(obs)


def test_gpu_config3_16384x30_off_policy():
    """Config 3 (16,384 envs x 30 assets, off-policy + device replay): collect from a
    resident series equals an independent env fed the gathered bars bit for bit, whose
    first 64 envs match the CPU oracle at every step; the
    replay's samples equal the numpy restatement of replay/buffer.py:39-79 on a
    512-sample subset; no sample crosses the reset between two collects; evaluate."""
    from pmenv import MarketSeries, TradingEnv
    from pmenv.off_policy import OffPolicy
    from oracle import replay_gather
    B, N, W, T, steps, cap = 16384, 30, 50, 1000, 64, 160
    rng = np.random.default_rng(33)
    closes = 100 * np.exp(np.cumsum(0.01 * rng.standard_normal((T, N)), axis=0))
    bars = np.stack([closes * np.exp(0.002 * rng.standard_normal((T, N))) for _ in range(3)] + [closes], -1)
    bars = bars.astype(np.float32)
    m = MarketSeries(bars, device=DEV)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV)
    acts = []
    gen = torch.Generator(device=DEV).manual_seed(3)

    def act(o):
        a = torch.softmax(torch.randn(B, N, device=DEV, generator=gen), -1)
        acts.append(a)
        return a

    seen = []
    loop = OffPolicy(env, m, capacity=cap, act=act, update=lambda *x: seen.append(len(x)), batch_size=1024,
                     generator=torch.Generator().manual_seed(4))
    start = m.random_starts(B, W, steps, generator=torch.Generator().manual_seed(5))
    rewards, obs = loop.collect(start, steps, random=True)           # collect_rand (off_policy.py:60-71)
    rewards, obs = loop.collect(start, steps)                         # _collect with the agent (:73-86)
    ref = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV)
    robs = m.initial_window(start, W)
    track = _OracleTrack(robs, 64, N, W)
    ref.reset(robs)
    st = start.long()
    for t in range(steps):
        bar = m.bars[st + W + t].contiguous()
        r, _ = ref.step(acts[t], robs, bar=bar)
        assert torch.equal(r, rewards[t]), f"step {t}"
        track.step(acts[t], bar, r, ref.value)
    assert torch.equal(robs, obs) and torch.equal(ref.value, env.value)
    track.window(obs)
    del ref, robs
    rb = loop.replay
    assert len(rb) == 2 * steps
    h0, e = rb.indices(8192, generator=torch.Generator().manual_seed(6))
    s, a, r, s2 = rb.gather(h0, e)
    rows = (h0.long().cpu()[:, None] + torch.arange(W + 1)[None, :]) % rb.H
    eps = torch.tensor(rb._row_ep)[rows]
    assert bool((eps == eps[:, :1]).all())                            # one episode per window
    pick = np.sort(np.random.default_rng(7).choice(8192, 512, replace=False))
    es, ea, er, es2 = replay_gather(bars, rb.days.cpu().numpy(), rb.actions.cpu().numpy(), rb.rewards.cpu().numpy(),
                                    h0.cpu().numpy()[pick], e.cpu().numpy()[pick], W)
    assert np.array_equal(s.cpu().numpy()[pick], es, equal_nan=True)
    assert np.array_equal(s2.cpu().numpy()[pick], es2, equal_nan=True)
    assert np.array_equal(a.cpu().numpy()[pick, :, 0], ea) and np.array_equal(r.cpu().numpy()[pick, 0, 0], er)
    del s, s2
    out = loop.update(4)
    assert len(out) == 4 and seen == [4] * 4
    met = loop.evaluate(start, 40, act=lambda o: torch.full((B, N), 1.0 / N, device=DEV))
    assert torch.equal(met["final_value"], env.value)
    for k in ("sharpe", "sortino", "max_drawdown", "average_turnover"):
        assert bool(torch.isfinite(met[k]).all()), k


def test_gpu_config2_4096x30_on_policy():
    """Config 2 (4,096 envs x 30 assets, A2C on-policy): the rollout with the env
    advancing straight into the device rollout buffer equals an independent in-place
    env bit for bit (rewards, values, windows), its rewards match the CPU oracle on a
    64-env sample, one update pass moves the policy, and the critic path (GAE over the
    stored rewards -> globally normalised advantages) runs on the HIP scan and moments."""
    from pmenv import TradingEnv, synth
    from pmenv.on_policy import OnPolicy, WindowCritic, WindowPolicy
    from oracle import gae as or_gae
    B, N, W, T = 4096, 30, 50, 32
    torch.manual_seed(0)
    ser = synth.series(W + T, B, N, seed=21, device=DEV)
    obs0 = synth.window_from_series(ser, W)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV)
    policy = WindowPolicy(W).to(DEV)
    loop = OnPolicy(env, policy, horizon=T, batch_size=4096, generator=torch.Generator().manual_seed(2))
    rewards = loop.rollout(obs0, ser[W:])
    buf = loop.buf
    ref = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV)
    robs = obs0.clone()
    ref.reset(robs)
    for t in range(1, T + 1):
        r, _ = ref.step(buf.a[t].contiguous(), robs, bar=ser[W + t - 1])
        assert torch.equal(r, rewards[t - 1]) and torch.equal(r, buf.r[t]), f"step {t}"
        assert torch.equal(robs, buf.obs(t)), f"window {t}"
        assert torch.equal(ref.value, buf.v[t])
    del ref, robs
    track = _OracleTrack(obs0, 64, N, W)                  # the rollout handle's own first 64 envs
    for t in range(1, T + 1):
        track.step(buf.a[t], ser[W + t - 1], buf.r[t], buf.v[t])
        track.window(buf.obs(t))
    w0 = [q.detach().clone() for q in policy.parameters()]
    losses = loop.update()
    assert losses.numel() == T and bool(torch.isfinite(losses).all())
    assert any(not torch.equal(a, b) for a, b in zip(w0, policy.parameters()))
    critic = WindowCritic(W).to(DEV)
    adv, ret, values = loop.advantages(critic, 0.99, 0.95)
    assert adv.shape == (T, B) and values.shape == (T + 1, B)
    oadv, oret = or_gae(buf.r[1:].cpu().numpy(), values.cpu().numpy(), None, 0.99, 0.95)
    np.testing.assert_allclose(ret.cpu().numpy(), oret, rtol=1e-5, atol=1e-5)
    z = (oadv - oadv.astype(np.float64).mean()) / (oadv.astype(np.float64).std() + 1e-8)
    np.testing.assert_allclose(adv.cpu().numpy(), z, rtol=1e-4, atol=1e-4)
    opt = torch.optim.Adam(critic.parameters(), lr=1e-3)
    cl = loop.update_critic(critic, opt, ret, batch_size=8192, generator=torch.Generator().manual_seed(3))
    assert cl.numel() == T * B // 8192 and bool(torch.isfinite(cl).all())


def test_gpu_config4_65536x30_sharded_eight_ways():
    """Config 4 (65,536 envs x 30 assets over 8 GPUs) as the bench shards it: each of the 8
    per-GPU shares (8,192 envs, global ids g * 8,192 .., its own Philox slice of the series
    — an Infinity-Cache-resident window on its own step path) run as its own handle equals
    the unsharded 65,536-env handle (the BASELINE one-launch step) bit for bit — rewards,
    values, windows — past the ring wrap, and the shares' first 64 envs match the CPU
    oracle at every step. Sharding is by construction exchange-free."""
    from pmenv import TradingEnv, synth
    from pmenv.parallel import shard_range
    G, Btot, N, W, T = 8, 65536, 30, 50, 56
    ser = synth.series(W + T, Btot, N, seed=41, device=DEV)
    act = synth.actions(T, Btot, N, seed=42, device=DEV)
    full = TradingEnv(num_envs=Btot, num_assets=N, window=W, device=DEV)
    fobs = synth.window_from_series(ser, W)
    full.reset(fobs)
    fr = torch.empty(T, Btot, device=DEV)
    for t in range(T):
        fr[t] = full.step(act[t], fobs, bar=ser[W + t])[0]
    paths = set()
    for g in range(G):
        lo, hi = shard_range(Btot, g, G)
        B = hi - lo
        sser = synth.series(W + T, B, N, env_offset=lo, seed=41, device=DEV)
        sact = synth.actions(T, B, N, env_offset=lo, seed=42, device=DEV)
        assert torch.equal(sser, ser[:, lo:hi]) and torch.equal(sact, act[:, lo:hi])   # the rank's own slice
        env = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV)
        paths.add(env.step_path.split(" | ")[-1])
        obs = synth.window_from_series(sser, W)
        track = _OracleTrack(obs, 64, N, W) if g in (0, G - 1) else None
        env.reset(obs)
        for t in range(T):
            r, _ = env.step(sact[t], obs, bar=sser[W + t])
            assert torch.equal(r, fr[t, lo:hi]), f"shard {g} step {t}: rewards"
            if track:
                track.step(sact[t], sser[W + t], r, env.value)
        assert torch.equal(obs, fobs[lo:hi]), f"shard {g}: windows"
        assert torch.equal(env.value, full.value[lo:hi]), f"shard {g}: values"
        if track:
            track.window(obs)
        del env, obs, sser, sact
    print(f"config 4 share path: {sorted(paths)}; unsharded: {full.step_path.split(' | ')[-1]}")
