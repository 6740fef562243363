"""Host-side logic that needs no GPU: config validation, sharding, the wrapper's
shape checks, and the bench's algorithmic byte model."""
import numpy as np
import pytest

from pmenv.config import EnvConfig
from pmenv.parallel import shard_range


def test_config_validation():
    EnvConfig(num_envs=4, num_assets=30, window=50).validate()
    with pytest.raises(ValueError):
        EnvConfig(reward="sharpe").validate()
    with pytest.raises(ValueError):
        EnvConfig(close_channel=4, features=5).validate()
    with pytest.raises(ValueError):
        EnvConfig(commission=1.5).validate()
    with pytest.raises(ValueError):
        EnvConfig(num_envs=0).validate()
    c = EnvConfig(reward="diff_sharpe", ring="chrono", norm="or", ret="net").to_c()
    assert (c.reward_kind, c.ring_mode, c.norm_mode, c.ret_mode) == (3, 1, 1, 1)


@pytest.mark.parametrize("G,world", [(65536, 8), (10, 3), (7, 8), (1, 1)])
def test_shard_range_partitions(G, world):
    spans = [shard_range(G, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == G
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c and a <= b
    assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


def test_bench_byte_model():
    import bench
    # B_step = 8*N*W*F + 20
    assert bench.step_bytes(30, 50, 5) == 60020
    assert bench.step_bytes(500, 50, 5) == 1000020
    assert bench.step_bytes(5, 50, 5) == 10020


def test_wrapper_refuses_cpu_device():
    from pmenv import TradingEnv
    with pytest.raises(ValueError):
        TradingEnv(num_envs=2, num_assets=5, window=8, device="cpu")


def test_device_replay_ring_indices_cpu():
    """DeviceReplay.add/indices host logic (replay/buffer.py:23-51) without a GPU."""
    import types
    import torch
    from pmenv.replay import DeviceReplay
    B, N, W, H = 3, 2, 4, 10
    rb = DeviceReplay(B, N, W, H, types.SimpleNamespace(device=torch.device("cpu")))
    with pytest.raises(ValueError):
        rb.indices(4)
    for k in range(H + 3):                              # wraps: oldest recorded step is k=3
        rb.add(torch.full((B,), k, dtype=torch.int32), torch.full((B, N), float(k)), torch.full((B,), float(k)))
    assert len(rb) == H and rb.head == 3
    h0, env = rb.indices(500, generator=torch.Generator().manual_seed(0))
    # every sample's W+1 consecutive steps are recorded and in chronological order
    ks = torch.stack([rb.days[(h0.long() + t) % H, env.long()] for t in range(W + 1)], 1)
    assert torch.all(ks[:, 1:] - ks[:, :-1] == 1) and ks.min() >= 3 and ks.max() <= H + 2
    assert set(env.tolist()) == set(range(B))
    with pytest.raises(ValueError):
        DeviceReplay(B, N, W, W + 1, None)


def test_rollout_buffer_sampling_host_logic():
    """DeviceRolloutBuffer's indexing (no GPU needed: the buffer is plain torch storage):
    every (step, env) pair of a rollout is sampled exactly once per pass, and a sample
    carries the window the action was taken on, the previous value / action and the
    close relative of its step (replay/rollout_buffer.py:103-142)."""
    import torch
    from pmenv.rollout_buffer import DeviceRolloutBuffer
    B, N, W, T = 5, 3, 4, 6
    buf = DeviceRolloutBuffer(B, N, W, T, device="cpu")
    g = torch.Generator().manual_seed(0)
    obs0 = torch.rand(B, N, W, 5, generator=g) + 0.5
    buf.reset(obs0)
    assert torch.equal(buf.obs(0), obs0) and bool((buf.a[0, :, 0] == 1).all()) and bool((buf.v[0] == 25000).all())
    for t in range(1, T + 1):
        buf.obs(t).copy_(torch.rand(B, N, W, 5, generator=g) + 0.5)
        buf.add(torch.full((B, N), float(t)), torch.full((B,), 1000.0 + t, dtype=torch.float64), torch.full((B,), -t))
    assert len(buf) == T
    with pytest.raises(IndexError):
        buf.add(torch.zeros(B, N), torch.zeros(B), torch.zeros(B))
    seen = []
    for s, a, r, v_prev, a_prev, p in buf.sample_random(10, generator=torch.Generator().manual_seed(1)):
        assert s.shape == (10, N, W, 5) and a.shape == (10, N, 1) and r.shape == (10, 1, 1)
        assert v_prev.shape == (10, 1, 1) and a_prev.shape == (10, N, 1) and p.shape == (10, N, 1)
        t = a[:, 0, 0].long()                                  # step index, as filled above
        assert torch.equal(r[:, 0, 0], -t.float())
        assert torch.equal(v_prev[:, 0, 0], torch.where(t == 1, 25000.0, 1000.0 + t - 1).float())
        env = torch.tensor([next(e for e in range(B) if torch.equal(s[i], buf.s[t[i] - 1, e])) for i in range(10)])
        assert torch.equal(p[..., 0], buf.s[t, env][..., W - 1, 3] / buf.s[t - 1, env][..., W - 1, 3])
        seen += list(zip(t.tolist(), env.tolist()))
    assert len(seen) == len(set(seen)) == T * B              # a permutation of all pairs
    ordered = [tuple(x) for s, a, *_ in buf.sample(B) for x in zip(a[:, 0, 0].long().tolist(), range(B))]
    assert ordered == [(t, e) for t in range(1, T + 1) for e in range(B)]


def test_off_policy_host_checks_cpu():
    """pmenv.off_policy.OffPolicy host logic (train/off_policy.py shape) without a GPU:
    series/env shape agreement, the replay sized from the env, the series-length check
    of collect, and the random seeding action being a simplex point."""
    import types
    import numpy as np
    import torch
    from pmenv.config import EnvConfig
    from pmenv.data import MarketSeries
    from pmenv.off_policy import OffPolicy
    cfg = EnvConfig(num_envs=4, num_assets=3, window=5)
    env = types.SimpleNamespace(cfg=cfg, device=torch.device("cpu"))
    bars = np.ones((40, 3, 4), np.float32)
    m = MarketSeries(bars, device="cpu")
    with pytest.raises(ValueError):
        OffPolicy(env, MarketSeries(np.ones((40, 2, 4), np.float32), device="cpu"), capacity=10)
    loop = OffPolicy(env, m, capacity=10)
    assert loop.replay.days.shape == (10, 4) and loop.replay.actions.shape == (10, 4, 3)
    with pytest.raises(ValueError):                      # 30 + 5 + 10 > 40 days
        loop.collect(torch.full((4,), 30, dtype=torch.int32), 10)
    a = loop._random_action()
    assert a.shape == (4, 3) and torch.all(a >= 0) and torch.allclose(a.sum(-1), torch.ones(4))


def test_gae_refuses_host_rewards():
    """A host tensor would hand the kernel a host pointer: refused before any launch."""
    import torch
    from pmenv import rollout
    with pytest.raises(ValueError):
        rollout.gae(torch.zeros(4, 3), torch.zeros(5, 3))
    with pytest.raises(ValueError):
        rollout.gae(torch.zeros(4, 3), torch.zeros(4, 3))          # values must be [T+1, B]
    with pytest.raises(ValueError):
        rollout.moments(torch.zeros(7))


def test_replay_valid_starts_stay_inside_one_episode():
    """The replay samples W+1 consecutive rows of one episode (buffer.py:17-21 keeps
    every epoch in its own row): starts whose window crosses a reset are excluded, on
    a wrapped ring too."""
    from pmenv.replay import valid_starts
    W, H = 3, 10
    # rows 0..9 written in order; episodes 0 (rows 0-5) then 1 (rows 6-9), oldest = 0
    ep = [0] * 6 + [1] * 4
    assert list(valid_starts(ep, 0, 10, W, H)) == [0, 1, 2]
    # the same ring after 4 more adds of episode 2 (rows 0-3 overwritten, oldest = 4)
    ep = [2] * 4 + [0, 0, 1, 1, 1, 1]
    got = list(valid_starts(ep, 4, 10, W, H))            # st counts from the oldest row (row 4)
    for st in got:
        rows = [(4 + st + i) % H for i in range(W + 1)]
        assert len({ep[r] for r in rows}) == 1
    assert got == [2]                                      # rows 6..9 are the only whole window
    one = valid_starts([5] * H, 0, H, W, H)               # one episode: every start, no scan
    assert isinstance(one, range) and list(one) == list(range(H - W - 1))
    # the vectorised scan against the per-start definition on random rings
    rng = np.random.default_rng(0)
    for _ in range(200):
        H = int(rng.integers(W + 2, 40))
        count = int(rng.integers(0, H + 1))
        oldest = int(rng.integers(0, H))
        chrono = np.sort(rng.integers(0, 4, count))        # ids grow along the ring
        ring = np.zeros(H, dtype=np.int64)
        ring[(oldest + np.arange(count)) % H] = chrono
        want = [st for st in range(max(count - W - 1, 0)) if ring[(oldest + st) % H] == ring[(oldest + st + W) % H]]
        assert list(valid_starts(ring, oldest, count, W, H)) == want
