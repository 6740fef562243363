"""Multi-GPU: envs shard embarrassingly across ranks (one process per GPU).

The env step itself has no cross-env coupling, so the env path's only exchange is the
advantage-normalisation moments {count, sum, sum of squares} (24 bytes, f64) —
one all-reduce per policy update over RCCL/xGMI (backend "nccl"), or gloo on CPU.
A policy replicated over the ranks adds one gradient all-reduce per optimizer step
(allreduce_grads: every parameter's gradient in one flat bucket).
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


def world(group=None):
    """Ranks in the default (or given) process group; 1 without torch.distributed."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group)
    return 1


def allreduce_grads(params, loss_sum, count, group=None):
    """Average replicated parameters' gradients over every rank's samples: the per-rank
    gradient SUMS, the loss sum and the sample count go through ONE all-reduce (a flat
    f64 bucket: the gradients of a small policy are a few hundred KB, one latency-bound
    exchange over xGMI), then every gradient is divided by the global count. Returns
    (global loss sum, global count) as python floats."""
    # every parameter, in order, on every rank: a parameter without a gradient here (a rank
    # with no envs, a branch unused there) contributes zeros, so the buckets line up over
    # ranks, and a has-gradient flag per parameter rides in the same bucket: a gradient is
    # written back only to trainable parameters some rank produced one for, so frozen or
    # unused parameters keep grad None and optimizers skip them as they would on one rank
    ps = list(params)
    if not ps:
        raise ValueError("allreduce_grads needs the replicated parameters")
    dev = ps[0].device
    # only trainable parameters count: a frozen one's local .grad neither rides in the bucket nor
    # gets a flag, and it is cleared on every rank alike (no rank keeps an un-averaged gradient)
    live = [p.requires_grad and p.grad is not None for p in ps]
    parts = [(p.grad.detach().reshape(-1) if ok else torch.zeros(p.numel(), device=p.device))
             .to(device=dev, dtype=torch.float64) for p, ok in zip(ps, live)]
    has = torch.tensor([1.0 if ok else 0.0 for ok in live], dtype=torch.float64, device=dev)
    extra = torch.stack([torch.as_tensor(loss_sum, dtype=torch.float64).reshape(()).to(dev),
                         torch.tensor(float(count), dtype=torch.float64, device=dev)])
    bucket = torch.cat(parts + [has, extra])
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(bucket, op=dist.ReduceOp.SUM, group=group)
    total, n = float(bucket[-2]), float(bucket[-1])
    flags = bucket[-2 - len(ps):-2].tolist()
    off = 0
    for p, f in zip(ps, flags):
        k = p.numel()
        if not p.requires_grad:
            p.grad = None
        elif f > 0:
            g = (bucket[off:off + k] / n).reshape(p.shape).to(device=p.device, dtype=p.dtype)
            if p.grad is None:
                p.grad = g
            else:
                p.grad.copy_(g)
        off += k
    return total, n
