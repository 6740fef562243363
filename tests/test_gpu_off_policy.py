"""The off-policy caller around the env step on an MI355X: train/off_policy.py's
collect -> update -> evaluate loop (pmenv.off_policy) with every env trading one
HBM-resident series, the steps recorded in the device replay and sampled back through
the HIP gather. Needs a GPU."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(DEV)


@pytest.mark.parametrize("B,N,W,steps,cap", [(64, 30, 20, 60, 80), (300, 7, 6, 40, 25)])
def test_gpu_off_policy_collect_update_evaluate(B, N, W, steps, cap):
    from pmenv import MarketSeries, TradingEnv
    from pmenv.off_policy import OffPolicy
    from oracle import replay_gather
    rng = np.random.default_rng(B + N)
    T = 400
    bars = (100 * np.exp(0.01 * rng.standard_normal((T, N, 4)).cumsum(0))).astype(np.float32)
    m = MarketSeries(bars, device=DEV)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV)
    seen, acts = [], []
    gen = torch.Generator(device=DEV).manual_seed(7)

    def act(o):                                 # a stand-in agent.act: random simplex, logged
        assert o.shape == (B, N, W, 5)
        a = torch.softmax(torch.randn(B, N, device=DEV, generator=gen), -1)
        acts.append(a)
        return a

    loop = OffPolicy(env, m, capacity=cap, act=act, update=lambda s, a, r, s_: seen.append((s, a, r, s_)),
                     batch_size=33, generator=torch.Generator().manual_seed(3))
    start = m.random_starts(B, W, steps, generator=torch.Generator().manual_seed(1))
    rewards, obs = loop.collect(start, steps)
    rb = loop.replay
    assert rewards.shape == (steps, B) and len(rb) == min(steps, cap) and len(acts) == steps
    for t in range(max(0, steps - cap), steps):   # the ring keeps the last `cap` steps
        assert torch.equal(rb.actions[t % cap], acts[t]) and torch.equal(rb.rewards[t % cap], rewards[t])

    # the same actions replayed on an independent env fed the same bars (bar mode) give
    # the same rewards, values and window, bit for bit
    ref = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV)
    robs = m.initial_window(start, W)
    ref.reset(robs)
    st = start.long()
    for t in range(steps):
        r, _ = ref.step(acts[t], robs, bar=m.bars[st + W + t].contiguous())
        assert torch.equal(r, rewards[t])
    assert torch.equal(robs, obs) and torch.equal(ref.value, env.value)
    # random seeding (collect_rand) runs too
    r0, _ = loop.collect(start, 3, random=True)
    assert r0.shape == (3, B) and torch.isfinite(r0).all()
    rewards, obs = loop.collect(start, steps)     # back to the logged run's state
    acts.clear()

    # the replay's window pair around the last recorded step: s ends on the day the last
    # action was taken on, s' is the env's current window (market channels)
    h0 = torch.full((B,), (rb.head - W) % cap, dtype=torch.int32, device=DEV)
    envs = torch.arange(B, dtype=torch.int32, device=DEV)
    s, a, r, s2 = rb.gather(h0, envs)
    assert torch.equal(s2[..., :4], obs[..., :4])
    assert torch.equal(s[..., 1:, :4], obs[..., :-1, :4])
    assert torch.equal(r[:, 0, 0], rewards[-1])

    # sampled batches equal the numpy restatement of replay/buffer.py:39-79
    out = loop.update(3)
    assert len(out) == 3 and len(seen) == 3
    h0, e = rb.indices(50, generator=torch.Generator().manual_seed(4))
    s, a, r, s2 = rb.gather(h0, e)
    es, ea, er, es2 = replay_gather(bars, rb.days.cpu().numpy(), rb.actions.cpu().numpy(), rb.rewards.cpu().numpy(),
                                    h0.cpu().numpy(), e.cpu().numpy(), W)
    assert np.array_equal(s.cpu().numpy(), es, equal_nan=True) and np.array_equal(s2.cpu().numpy(), es2, equal_nan=True)
    assert np.array_equal(a.cpu().numpy()[..., 0], ea) and np.array_equal(r.cpu().numpy()[:, 0, 0], er)
    for s_, a_, r_, sn_ in seen:
        assert s_.shape == (33, N, W, 5) and sn_.shape == s_.shape and a_.shape == (33, N, 1) and r_.shape == (33, 1, 1)

    # evaluation: per-env metrics over a deterministic run; final value = the env's value
    met = loop.evaluate(start, 30, act=lambda o: torch.full((B, N), 1.0 / N, device=DEV))
    assert torch.equal(met["final_value"], env.value)
    for k in ("sharpe", "sortino", "max_drawdown", "average_turnover"):
        assert torch.isfinite(met[k]).all(), k
    assert env.info is not None and len(env.info["values"]) == 31


def test_gpu_replay_windows_never_straddle_collect_calls():
    """Two collect calls from different start days into one replay ring: every sampled
    window's W+1 rows belong to one episode and hold consecutive days of one env
    (advisor finding: a window spanning the reset mixed two episodes' actions)."""
    from pmenv import MarketSeries, TradingEnv
    from pmenv.off_policy import OffPolicy
    B, N, W, T = 40, 7, 6, 300
    rng = np.random.default_rng(3)
    bars = (100 * np.exp(0.01 * rng.standard_normal((T, N, 4)).cumsum(0))).astype(np.float32)
    m = MarketSeries(bars, device=DEV)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV)
    loop = OffPolicy(env, m, capacity=50, batch_size=16)
    g = torch.Generator().manual_seed(5)
    loop.collect(m.random_starts(B, W, 30, generator=g), 30)
    loop.collect(m.random_starts(B, W, 30, generator=g), 30)   # a reset: a new episode in the same ring
    rb = loop.replay
    h0, e = rb.indices(4000, generator=torch.Generator().manual_seed(6))
    rows = (h0.long().cpu()[:, None] + torch.arange(W + 1)[None, :]) % rb.H
    eps = torch.tensor(rb._row_ep)[rows]
    assert bool((eps == eps[:, :1]).all())
    days = rb.days.cpu()[rows, e.long().cpu()[:, None]]
    assert bool((days[:, 1:] - days[:, :-1] == 1).all())
    assert len(set(eps[:, 0].tolist())) == 2                   # both episodes are sampled
