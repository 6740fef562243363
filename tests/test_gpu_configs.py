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


def _oracle_sample(ser, act, S, N, W, T, **cfg_kw):
    """The first S envs of a synthetic run through the CPU oracle and through a fresh
    HIP env of S envs, on identical inputs: rewards within |d| <= 1e-6 |r| + 1e-9,
    values rtol 1e-12, market channels bit-exact."""
    from pmenv import TradingEnv, synth
    from pmenv.config import EnvConfig
    sub = TradingEnv(num_envs=S, num_assets=N, window=W, device=DEV, **cfg_kw)
    sobs = synth.window_from_series(ser[:W, :S].contiguous(), W)
    cenv = OracleEnv(EnvConfig(num_envs=S, num_assets=N, window=W, **cfg_kw))
    cobs = sobs.cpu().numpy().copy()
    sub.reset(sobs)
    cenv.reset(cobs)
    ser_h, act_h = ser[:, :S].cpu().numpy(), act[:, :S].cpu().numpy()
    for t in range(T):
        gr, _ = sub.step(act[t, :S].contiguous(), sobs, bar=ser[W + t, :S].contiguous())
        cr, _, _ = cenv.step(act_h[t], cobs, bar=ser_h[W + t])
        g = gr.cpu().numpy().astype(np.float64)
        both_nan = np.isnan(g) & np.isnan(cr)
        err = np.where(both_nan, 0.0, np.abs(g - cr))
        assert np.all(err <= 1e-6 * np.abs(np.nan_to_num(cr)) + 1e-9), f"step {t}: reward err {err.max():.3e}"
        np.testing.assert_allclose(sub.value.cpu().numpy(), cenv.value, rtol=1e-12)
    o = sobs.cpu().numpy()
    assert np.array_equal(o[..., :4], cobs[..., :4])
    np.testing.assert_allclose(o[..., 4], cobs[..., 4], rtol=2e-7, atol=1e-12)


@pytest.mark.parametrize("commission", [0.0, 0.0025])
def test_gpu_config5_8192x500_diff_sharpe(commission):
    """Config 5 (8,192 envs x 500 assets x 50 days x 5, differential Sharpe) through the
    default in-place path past the ring wrap (T = 56 > W): every env's window equals
    the sliding series, the weight channel equals the ring (get_all), values and
    rewards are finite, and every env's reward equals a torch f64 restatement of the
    differential Sharpe recursion over its own returns (commission 0); a 64-env sample
    against the CPU oracle, with and without commission."""
    from pmenv import TradingEnv, synth
    B, N, W, T = 8192, 500, 50, 56
    ser = synth.series(W + T, B, N, seed=51, device=DEV)
    act = synth.actions(T, B, N, seed=52, device=DEV)
    obs = synth.window_from_series(ser, W)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, reward="diff_sharpe",
                     commission=commission, track_info=commission == 0.0)
    env.reset(obs)
    eta = env.cfg.sharpe_eta
    A = torch.zeros(B, dtype=torch.float64, device=DEV)
    Bm = torch.zeros(B, dtype=torch.float64, device=DEV)
    for t in range(T):
        r, _ = env.step(act[t], obs, bar=ser[W + t])
        assert bool(torch.isfinite(r).all()) and bool(torch.isfinite(env.value).all())
        if commission == 0.0:
            ret = env.info["returns"][-1]
            y = (ser[W + t, ..., 3] / ser[W + t - 1, ..., 3]).double()
            assert torch.allclose(ret, (act[t].double() * y).sum(-1), rtol=1e-12)
            R = ret - 1.0
            dA, dB, var = R - A, R * R - Bm, Bm - A * A
            ref = torch.where(var > 1e-12, (Bm * dA - 0.5 * A * dB) / (var * var.clamp(min=0).sqrt()),
                              torch.zeros_like(var))
            err = (r.double() - ref).abs()
            assert bool((err <= 1e-6 * ref.abs() + 1e-9).all()), f"step {t}: {float(err.max()):.3e}"
            A, Bm = A + eta * dA, Bm + eta * dB
    assert torch.equal(obs[..., :4], ser[T:T + W].permute(1, 2, 0, 3))
    assert torch.equal(obs[..., 4], env.weights.get_all())
    assert bool(env.weights.is_full.all()) and env.nonfinite_count() == 0
    del obs
    _oracle_sample(ser, act, 64, N, W, T, reward="diff_sharpe", commission=commission)


def test_gpu_config3_16384x30_off_policy():
    """Config 3 (16,384 envs x 30 assets, off-policy + device replay): collect from a
    resident series equals an independent env fed the gathered bars bit for bit; the
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
    ref.reset(robs)
    st = start.long()
    for t in range(steps):
        r, _ = ref.step(acts[t], robs, bar=m.bars[st + W + t].contiguous())
        assert torch.equal(r, rewards[t]), f"step {t}"
    assert torch.equal(robs, obs) and torch.equal(ref.value, env.value)
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
    _oracle_sample(ser, buf.a[1:].contiguous(), 64, N, W, T)
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
