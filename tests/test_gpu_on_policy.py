"""The on-policy caller around the env step on an MI355X: train/on_policy.py's
rollout -> update loop (pmenv.on_policy) with the env advancing its window straight
into the device rollout buffer, the batched A2C loss as the fused HIP op and the GAE
pass over the stored rewards. Needs a GPU."""
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


@pytest.mark.parametrize("B,N,W,T", [(64, 30, 20, 12), (1100, 8, 10, 6)])
def test_gpu_on_policy_rollout_and_update(B, N, W, T):
    from pmenv import TradingEnv, synth
    from pmenv.on_policy import OnPolicy, WindowPolicy
    from pmenv.rollout import gae
    torch.manual_seed(0)
    ser = synth.series(W + T, B, N, seed=5, device=DEV)
    obs0 = synth.window_from_series(ser, W)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV)
    policy = WindowPolicy(W).to(DEV)
    loop = OnPolicy(env, policy, horizon=T, batch_size=B, generator=torch.Generator().manual_seed(2))
    rewards = loop.rollout(obs0, ser[W:])
    buf = loop.buf
    assert len(buf) == T and rewards.shape == (T, B)
    # the same actions replayed on an independent env stepping in place give the same
    # rewards, values and windows, bit for bit
    ref = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV)
    robs = obs0.clone()
    ref.reset(robs)
    assert torch.equal(robs, buf.obs(0))
    for t in range(1, T + 1):
        r, _ = ref.step(buf.a[t].contiguous(), robs, bar=ser[W + t - 1])
        assert torch.equal(r, rewards[t - 1]) and torch.equal(r, buf.r[t])
        assert torch.equal(robs, buf.obs(t)), f"window {t}"
        assert torch.equal(ref.value, buf.v[t])
    # price relatives of a step == the series' close relative (the env's own fp32 quotient)
    p = buf.price_relatives(T)
    assert torch.equal(p, ser[W + T - 1, ..., 3] / ser[W + T - 2, ..., 3])
    # log-return reward == log(sum a * p) of the stored action and relative
    lr = torch.log((buf.a[T].double() * p.double()).sum(-1))
    assert torch.allclose(buf.r[T].double(), lr, rtol=1e-6, atol=1e-9)
    # one update pass over every (step, env): finite losses, the policy moves
    w0 = [q.detach().clone() for q in policy.parameters()]
    losses = loop.update()
    assert losses.numel() == T and bool(torch.isfinite(losses).all())
    assert any(not torch.equal(a, b) for a, b in zip(w0, policy.parameters()))
    # returns over the stored rollout == the standalone GAE pass on the same rewards
    values = torch.randn(T + 1, B, device=DEV)
    adv, ret = buf.returns(values, 0.99, 0.95)
    adv2, _ = gae(buf.r[1:].contiguous(), values, None, 0.99, 0.95)
    assert torch.equal(adv, adv2) and torch.allclose(ret, adv + values[:T], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("ring", ["storage", "chrono"])
# (the LDS-staged gather: 16-B granular windows of <= 64 KiB; the per-row gather: the rest)
@pytest.mark.parametrize("B,N,W,T", [(33, 7, 6, 20), (5, 30, 50, 60), (64, 1, 2, 9), (3, 80, 50, 8)])
def test_gpu_compact_rollout_rematerialises_the_env_windows(ring, B, N, W, T):
    """The compact rollout (resident series, O(T*B*N) storage) re-materialises, for
    every step t and env, exactly the window the env held after t steps — market
    channels from the series, the weight channel from the recorded w' in the ring's
    order (storage order past the wrap, T > W) — and the price relatives of the step."""
    from pmenv import MarketSeries, TradingEnv
    from pmenv.rollout_buffer import DeviceRolloutBuffer
    rng = np.random.default_rng(B + N + W)
    Ts = W + T + 40
    bars = (100 * np.exp(0.01 * rng.standard_normal((Ts, N, 4)).cumsum(0))).astype(np.float32)
    m = MarketSeries(bars, device=DEV)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, ring=ring)
    buf = DeviceRolloutBuffer(B, N, W, T, device=DEV, series=m, ring=ring)
    start = m.random_starts(B, W, T, generator=torch.Generator().manual_seed(1))
    buf.reset(start=start)
    obs = m.initial_window(start, W)
    env.reset(obs)
    assert torch.equal(buf.obs(0), obs)
    w = torch.empty(B, N, device=DEV)
    for t in range(1, T + 1):
        a = torch.softmax(torch.randn(B, N, device=DEV), -1)
        r, _ = env.step(a, obs, series=m, day=start + W + t - 1, weights_out=w)
        buf.add(a, env.value, r, weights=w)
        assert torch.equal(buf.obs(t), obs), f"window after {t} steps"
        assert torch.equal(buf.price_relatives(t), m.bars[start.long() + W + t - 1, :, 3] /
                           m.bars[start.long() + W + t - 2, :, 3])
    s, a_, r_, v_prev, a_prev, p = buf.gather(torch.tensor([T, 1, T // 2], device=DEV), torch.tensor([0, B - 1, B // 2],
                                                                                                    device=DEV))
    assert s.shape == (3, N, W, 5) and p.shape == (3, N, 1) and v_prev.shape == (3, 1, 1)
    assert buf.nbytes() < 4 * (T + 1) * B * N * 4 + 64 * B      # O(T * B * N): no windows kept
    # a C caller's misaligned output view (4 B past a 16-B boundary) takes the dword row
    # form instead of the tile's 16-B stores: the same windows
    import ctypes
    from pmenv import _abi
    ti = torch.tensor([T, 1, T // 2], dtype=torch.int32, device=DEV)
    ei = torch.tensor([0, B - 1, B // 2], dtype=torch.int32, device=DEV)
    raw = torch.full((3 * N * W * 5 + 4,), -1.0, device=DEV)
    mis = raw[1:1 + 3 * N * W * 5]
    assert mis.data_ptr() % 16 == 4
    st = ctypes.c_void_p(torch.cuda.current_stream(DEV).cuda_stream)
    pp = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    _abi.check(_abi.load().pmenv_rollout_gather(pp(m.bars), m.bars.shape[0], N, 5, W, pp(buf.start), pp(buf.w), T, B,
                                                _abi.RING_MODES[ring], pp(ti), pp(ei), 3, pp(mis), st))
    assert torch.equal(mis.view(3, N, W, 5), buf.windows(ti, ei))
    assert bool((raw[0] == -1.0) & (raw[-3:] == -1.0).all())         # nothing written outside the view


def test_gpu_on_policy_compact_loop():
    """OnPolicy over a resident series with the compact buffer: the rewards equal an
    independent env fed the gathered bar batch bit for bit, an update pass and the
    critic's GAE / normalised advantages run on re-materialised windows."""
    from pmenv import MarketSeries, TradingEnv
    from pmenv.on_policy import OnPolicy, WindowCritic, WindowPolicy
    B, N, W, T, Ts = 256, 30, 50, 24, 400
    rng = np.random.default_rng(7)
    bars = (100 * np.exp(0.01 * rng.standard_normal((Ts, N, 4)).cumsum(0))).astype(np.float32)
    m = MarketSeries(bars, device=DEV)
    torch.manual_seed(1)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV)
    policy = WindowPolicy(W).to(DEV)
    loop = OnPolicy(env, policy, horizon=T, series=m, batch_size=B, generator=torch.Generator().manual_seed(2))
    start = m.random_starts(B, W, T, generator=torch.Generator().manual_seed(3))
    rewards = loop.rollout(start=start)
    buf = loop.buf
    assert buf.compact and rewards.shape == (T, B)
    ref = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV)
    robs = m.initial_window(start, W)
    ref.reset(robs)
    for t in range(1, T + 1):
        r, _ = ref.step(buf.a[t].contiguous(), robs, bar=m.bars[start.long() + W + t - 1].contiguous())
        assert torch.equal(r, rewards[t - 1]) and torch.equal(ref.value, buf.v[t])
    assert torch.equal(robs, loop.obs) and torch.equal(buf.obs(T), robs)
    w0 = [q.detach().clone() for q in policy.parameters()]
    losses = loop.update()
    assert losses.numel() == T and bool(torch.isfinite(losses).all())
    assert any(not torch.equal(a, b) for a, b in zip(w0, policy.parameters()))
    critic = WindowCritic(W).to(DEV)
    adv, ret, values = loop.advantages(critic)
    assert adv.shape == (T, B) and bool(torch.isfinite(adv).all())
    assert abs(float(adv.mean())) < 1e-4 and abs(float(adv.std(unbiased=False)) - 1.0) < 1e-3


# ---------------------------------------------------------------- actor-critic, two ranks
AC = dict(G=1001, N=30, W=50, T=8)


def _ac_run(lo, hi, dev, group=None):
    """OnPolicy over global envs [lo, hi): an exploring rollout (noise keyed by global env
    id), the critic's GAE advantages normalised over every rank (the HIP moments + the
    24-byte all-reduce), one update_actor_critic (one gradient all-reduce). f64 policy and
    critic, so the ranks' sums differ from the unsharded run's by reassociation only."""
    from pmenv import TradingEnv, synth
    from pmenv.on_policy import OnPolicy, WindowCritic, WindowPolicy
    G, N, W, T = AC["G"], AC["N"], AC["W"], AC["T"]
    B = hi - lo
    ser = synth.series(W + T, B, N, env_offset=lo, seed=42, device=dev)
    obs0 = synth.window_from_series(ser, W)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=dev)
    torch.manual_seed(0)
    policy = WindowPolicy(W).double().to(dev)
    critic = WindowCritic(W).double().to(dev)
    loop = OnPolicy(env, policy, horizon=T, explore_std=0.3, env_offset=lo)
    loop.optim = torch.optim.SGD(policy.parameters(), lr=1e-2)
    rewards = loop.rollout(obs0, ser[W:])
    adv, ret, values = loop.advantages(critic, group=group)
    loss = loop.update_actor_critic(adv, group=group, chunk=2048)
    return (rewards.cpu(), [p.detach().cpu() for p in policy.parameters()],
            [p.grad.detach().cpu() for p in policy.parameters()], loss)


def _ac_worker(rank, world, port, root, q):
    import os
    import sys
    for p in (os.path.join(root, "pm-rl_amd"), os.path.join(root, "oracle")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        from pmenv import parallel
        lo, hi = parallel.shard_range(AC["G"], rank, world)
        r, params, grads, loss = _ac_run(lo, hi, dev)
        q.put((rank, lo, hi, r.numpy(), [p.numpy() for p in params], [g.numpy() for g in grads], loss))
    finally:
        dist.destroy_process_group()


def test_gpu_actor_critic_two_ranks_equal_unsharded_update():
    """The normalised advantages feed a loss: two gloo ranks (spawned, both on cuda:0), each
    stepping half of the envs, take the same actor-critic update as one unsharded run —
    the rollouts bit for bit, the averaged gradients and the parameters to f64
    reassociation."""
    import os
    import socket
    import torch.multiprocessing as mp
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ac_worker, args=(r, 2, port, root, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    r_full, params, grads, loss = _ac_run(0, AC["G"], DEV)
    for rank, lo, hi, r, ps, gs, l in res:
        assert np.array_equal(r, r_full.numpy()[:, lo:hi]), f"rank {rank}: rollout rewards"
        assert abs(l - loss) <= 1e-10 * abs(loss), f"rank {rank}: loss {l} vs {loss}"
        gmax = max(float(g.abs().max()) for g in grads)
        for i, (x, y) in enumerate(zip(gs, grads)):
            np.testing.assert_allclose(x, y.numpy(), rtol=1e-9, atol=1e-11 * gmax, err_msg=f"rank {rank} grad {i}")
        for i, (x, y) in enumerate(zip(ps, params)):
            np.testing.assert_allclose(x, y.numpy(), rtol=1e-12, atol=1e-13, err_msg=f"rank {rank} param {i}")
