"""Multi-GPU: envs shard embarrassingly across ranks (one process per GPU).

The env step itself has no cross-env coupling, so the only exchange is the
advantage-normalisation moments {count, sum, sum of squares} (24 bytes, f64) —
one all-reduce per policy update over RCCL/xGMI (backend "nccl"), or gloo on CPU.
"""
import torch
import torch.distributed as dist


def shard_range(global_envs, rank, world):
    """Contiguous env block [lo, hi) owned by `rank` (remainder spread over the first ranks)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, rem = divmod(int(global_envs), int(world))
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def allreduce_moments(local, group=None):
    """Sum per-rank {count, sum, sumsq} f64 moments across ranks (in place) and
    return (count, mean, var) as python floats (population variance)."""
    t = local if local.dtype == torch.float64 else local.to(torch.float64)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    n, s, q = (float(v) for v in t.tolist())
    mean = s / n if n > 0 else 0.0
    var = max(q / n - mean * mean, 0.0) if n > 0 else 0.0
    return n, mean, var


def local_moments_cpu(x):
    """CPU/host counterpart of rollout.moments (for gloo paths and tests)."""
    x = x.detach().to("cpu", torch.float64).reshape(-1)
    return torch.stack([torch.tensor(float(x.numel()), dtype=torch.float64), x.sum(), (x * x).sum()])


def normalize(adv, group=None, eps=1e-8):
    """Global advantage normalisation: local moments -> all-reduce -> (adv - mean) / std."""
    if adv.is_cuda:
        from .rollout import moments
        m = moments(adv)
    else:
        m = local_moments_cpu(adv)
    _, mean, var = allreduce_moments(m, group)
    return (adv - mean) / (var ** 0.5 + eps)
