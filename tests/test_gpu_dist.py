"""Multi-rank readiness of the product path on a GPU: two ranks (fresh spawned
processes, gloo, both on cuda:0 — RCCL refuses two ranks on one device) each run
pmenv.TradingEnv on their shard_range slice of a BASELINE-shaped batch and normalise
their rewards with pmenv.parallel.normalize (the HIP moments kernel + the 24-byte
all-reduce). The shards' rewards, values and windows equal one unsharded run bit
for bit; the all-reduced moments equal the unsharded ones. Needs a GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

G, N, W, T = 3001, 30, 50, 60          # odd total: the shards differ in size


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(lo, hi, dev, impl="auto"):
    """Rank work: the global envs [lo, hi) of the synthetic BASELINE workload."""
    from pmenv import TradingEnv, synth
    B = hi - lo
    ser = synth.series(W + T, B, N, env_offset=lo, seed=42, device=dev)
    act = synth.actions(T, B, N, env_offset=lo, seed=43, device=dev)
    obs = synth.window_from_series(ser, W)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=dev, step_impl=impl)
    env.reset(obs)
    rew = torch.stack([env.step(act[t], obs, bar=ser[W + t])[0] for t in range(T)])   # [T, B]
    return rew, env.value, obs


def _worker(rank, world, port, root, q, impl):
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
        from pmenv.rollout import moments
        lo, hi = parallel.shard_range(G, rank, world)
        rew, val, obs = _run(lo, hi, dev, impl)
        m = moments(rew)                                          # HIP moments kernel, [3] f64 on the GPU
        n, mean, var = parallel.allreduce_moments(m.clone())     # the 24-byte all-reduce
        z = parallel.normalize(rew)
        q.put((rank, lo, hi, rew.cpu().numpy(), val.cpu().numpy(), obs.cpu().numpy(), n, mean, var,
               z.cpu().numpy(), m.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("impl_shards,impl_full", [("auto", "auto"), ("flat", "two_launch")])
def test_gpu_sharded_ranks_equal_unsharded_run(impl_shards, impl_full):
    """("flat", "two_launch"): the ranks step with the one-launch flat kernel, the
    unsharded run with the two-launch path — still the same bits."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, root, q, impl_shards)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    dev = torch.device("cuda:0")
    from pmenv.rollout import moments
    rew, val, obs = _run(0, G, dev, impl_full)
    full = rew.cpu().numpy()
    fv, fo = val.cpu().numpy(), obs.cpu().numpy()
    m_full = moments(rew).cpu().numpy()
    n_tot = 0
    for rank, lo, hi, r, v, o, n, mean, var, z, m in res:
        assert np.array_equal(r, full[:, lo:hi]), f"rank {rank} rewards"
        assert np.array_equal(v, fv[lo:hi]), f"rank {rank} values"
        assert np.array_equal(o, fo[lo:hi]), f"rank {rank} windows"
        assert n == G * T
        assert np.isclose(mean, m_full[1] / m_full[0], rtol=1e-12, atol=1e-15)
        assert np.isclose(var, m_full[2] / m_full[0] - (m_full[1] / m_full[0]) ** 2, rtol=1e-9, atol=1e-18)
        np.testing.assert_allclose(z, (r - mean) / (var ** 0.5 + 1e-8), rtol=1e-5, atol=1e-6)
        n_tot += m[0]
    assert n_tot == G * T
    np.testing.assert_allclose(res[0][10][1:] + res[1][10][1:], m_full[1:], rtol=1e-12)


def _rccl_worker(port, root, q):
    import sys
    for p in (os.path.join(root, "pm-rl_amd"), os.path.join(root, "oracle")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)       # RCCL
    try:
        from pmenv import parallel
        from pmenv.rollout import moments
        rew, _, _ = _run(0, G, dev)
        z = parallel.normalize(rew)                               # HIP moments + RCCL all_reduce
        n, mean, var = parallel.allreduce_moments(moments(rew).clone())
        torch.manual_seed(0)
        lin = torch.nn.Linear(N, 1).to(dev).double()
        lin(rew.double().T[:, :N]).sum().backward()               # rewards [T = 60, B] -> B rows of N inputs
        before = [p.grad.clone() for p in lin.parameters()]
        total, cnt = parallel.allreduce_grads(list(lin.parameters()), torch.tensor(3.0, device=dev), 4.0)
        after = [p.grad.clone() for p in lin.parameters()]
        q.put((dist.get_backend(), z.cpu().numpy(), n, mean, var, total, cnt,
               [b.cpu().numpy() for b in before], [a.cpu().numpy() for a in after], rew.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def test_gpu_rccl_single_rank_collectives():
    """The RCCL branch ("nccl" backend) of the path's collectives, executed on the GPU with one
    rank (the one-GPU box cannot hold two RCCL ranks on one device): the advantage moments'
    all-reduce and normalisation, and the gradient bucket's all-reduce, equal the local
    computation."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), root, q))
    p.start()
    backend, z, n, mean, var, total, cnt, before, after, rew = q.get(timeout=240)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert backend == "nccl"
    x = rew.astype(np.float64)
    assert n == x.size
    assert np.isclose(mean, x.mean(), rtol=1e-12, atol=1e-15)
    assert np.isclose(var, x.var(), rtol=1e-9, atol=1e-18)
    np.testing.assert_allclose(z, (rew - mean) / (var ** 0.5 + 1e-8), rtol=1e-5, atol=1e-6)
    assert total == 3.0 and cnt == 4.0
    for b, a in zip(before, after):
        np.testing.assert_allclose(a, b / 4.0, rtol=1e-15)
