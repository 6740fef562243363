"""Multi-process path on CPU (gloo, world_size 2): env sharding is exact and the
advantage-moment all-reduce equals the single-process result."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, root, q):
    import sys
    for p in (os.path.join(root, "pm-rl_amd"), os.path.join(root, "oracle")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import OracleEnv, synth_series, synth_actions
    from pmenv.config import EnvConfig
    from pmenv.parallel import allreduce_moments, local_moments_cpu, normalize, shard_range

    G, N, W, T = 10, 6, 8, 12
    lo, hi = shard_range(G, rank, world)
    B = hi - lo
    ser = synth_series(W + T, B, N, env_offset=lo)
    act = synth_actions(T, B, N, env_offset=lo)
    obs = np.zeros((B, N, W, 5), np.float32)
    obs[..., :4] = ser[:W].transpose(1, 2, 0, 3)
    env = OracleEnv(EnvConfig(num_envs=B, num_assets=N, window=W))
    env.reset(obs)
    rewards = []
    for t in range(T):
        r, _, _ = env.step(act[t], obs, bar=ser[W + t])
        rewards.append(r)
    rew = torch.tensor(np.stack(rewards))                  # [T, B]
    n, mean, var = allreduce_moments(local_moments_cpu(rew))
    z = normalize(rew)
    q.put((rank, lo, hi, rew.numpy(), env.value.copy(), n, mean, var, z.numpy()))
    dist.destroy_process_group()


def test_sharded_envs_equal_unsharded_and_moments_allreduce():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, root, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle import OracleEnv, synth_series, synth_actions
    from pmenv.config import EnvConfig
    G, N, W, T = 10, 6, 8, 12
    ser = synth_series(W + T, G, N)
    act = synth_actions(T, G, N)
    obs = np.zeros((G, N, W, 5), np.float32)
    obs[..., :4] = ser[:W].transpose(1, 2, 0, 3)
    env = OracleEnv(EnvConfig(num_envs=G, num_assets=N, window=W))
    env.reset(obs)
    full = np.stack([env.step(act[t], obs, bar=ser[W + t])[0] for t in range(T)])
    for rank, lo, hi, rew, val, n, mean, var, z in res:
        assert np.array_equal(rew, full[:, lo:hi])          # bit-exact: envs are independent
        assert np.array_equal(val, env.value[lo:hi])
        x = full.astype(np.float64)
        assert n == x.size
        assert np.isclose(mean, x.mean(), rtol=1e-12, atol=1e-15)
        assert np.isclose(var, x.var(), rtol=1e-9, atol=1e-18)
        np.testing.assert_allclose(z, (full[:, lo:hi] - mean) / (var ** 0.5 + 1e-8), rtol=1e-5, atol=1e-6)
