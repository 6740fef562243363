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
