"""Trainer-side twin of the env step: the differentiable batched portfolio reward of
the PG / A2C agents, as a fused HIP forward + backward (libpmenv.so).

    reference                                   here
    PG._reward(a, _v, _a, p)   pg.py:40-82      pg_reward(a, _v, _a, p, reward=..., scale=...)
    A2C._loss(a, _v, _a, p)    a2c.py:40-82     a2c_loss(a, _v, _a, p, ...)  (= -pg_reward)

`a` [B, N, 1] (requires grad), `_v` [B, 1, 1], `p` [B, N, 1]; `_a` is accepted for
signature parity and unused, as in the reference with COMISSION = 0 (the reference's
commission branch raises TypeError, pg.py:62). The normalisation decision of the
reference is taken over the whole batch (`norm="global_or"`, pg.py:52).
"""
import ctypes

import torch

from . import _abi
from .config import REWARD, REWARD_SCALE

_KINDS = {"log_returns": 0, "returns": 1, "sharpe_ratio": 2}


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


class _BatchReward(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, v_prev, p, kind, norm, scale, want_ret):
        lib = _abi.load()
        B = a.shape[0]
        a2 = a.detach().reshape(B, -1).to(torch.float32).contiguous()
        N = a2.shape[1]
        v2 = v_prev.detach().reshape(B).to(device=a.device, dtype=torch.float32).contiguous()
        p2 = p.detach().reshape(B, N).to(device=a.device, dtype=torch.float32).contiguous()
        work = torch.empty(lib.pmenv_batch_reward_workspace(B) // 8, dtype=torch.float64, device=a.device)
        out = torch.empty((), dtype=torch.float32, device=a.device)
        ret = torch.empty(B, dtype=torch.float32, device=a.device) if want_ret else None
        s = ctypes.c_void_p(torch.cuda.current_stream(a.device).cuda_stream)
        _abi.check(lib.pmenv_batch_reward_forward(_p(a2), _p(v2), _p(p2), B, N, _KINDS[kind],
                                                  _abi.BATCH_NORM_MODES[norm], float(scale), _p(work),
                                                  _p(out), _p(ret) if ret is not None else None, s),
                   None, "pmenv_batch_reward_forward")
        ctx.save_for_backward(a2, v2, p2, work)
        ctx.kind, ctx.scale, ctx.shape = kind, scale, a.shape
        if ret is None:
            return out.to(a.dtype)
        ctx.mark_non_differentiable(ret)
        return out.to(a.dtype), ret

    @staticmethod
    def backward(ctx, grad_out, _grad_ret=None):
        lib = _abi.load()
        a2, v2, p2, work = ctx.saved_tensors
        B, N = a2.shape
        g = grad_out.detach().to(torch.float32).reshape(1).contiguous()
        grad_a = torch.empty_like(a2)
        s = ctypes.c_void_p(torch.cuda.current_stream(a2.device).cuda_stream)
        _abi.check(lib.pmenv_batch_reward_backward(_p(a2), _p(v2), _p(p2), B, N, _KINDS[ctx.kind],
                                                   float(ctx.scale), _p(work), _p(g), _p(grad_a), s),
                   None, "pmenv_batch_reward_backward")
        return grad_a.reshape(ctx.shape), None, None, None, None, None, None


def batch_reward(a, v_prev, p, reward=REWARD, scale=REWARD_SCALE, norm="global_or", return_ret=False):
    if reward not in _KINDS:
        raise ValueError(f"batched reward supports {sorted(_KINDS)}, got {reward!r}")
    if norm not in _abi.BATCH_NORM_MODES:
        raise ValueError(f"norm must be one of {sorted(_abi.BATCH_NORM_MODES)}")
    if not a.is_cuda:
        raise ValueError("pmenv batched reward runs on the GPU only (no CPU fallback)")
    if return_ret:
        return _BatchReward.apply(a, v_prev, p, reward, norm, scale, True)
    return _BatchReward.apply(a, v_prev, p, reward, norm, scale, False)


def pg_reward(a, _v, _a, p, reward=REWARD, scale=REWARD_SCALE, norm="global_or"):
    """PG._reward (agent/pg/pg.py:40-82)."""
    return batch_reward(a, _v, p, reward=reward, scale=scale, norm=norm)


def a2c_loss(a, _v, _a, p, reward=REWARD, scale=REWARD_SCALE, norm="global_or"):
    """A2C._loss (agent/a2c.py/a2c.py:40-82) = -PG._reward."""
    return -batch_reward(a, _v, p, reward=reward, scale=scale, norm=norm)
