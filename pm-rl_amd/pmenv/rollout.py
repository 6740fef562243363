"""Rollout returns on device.

The reference's replay/rollout_buffer.py stores (s, a, v, r) per day (:43-57) and
computes no returns; the north star asks for its GAE / discounted-return pass as
a device kernel. pmenv_gae_ex scans each env's column of a time-major [T, B]
rollout backwards (lanes = envs, coalesced rows; the horizon split over waves and,
for few envs, over workgroups).
"""
import ctypes

import torch

from . import _abi


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def gae(rewards, values, dones=None, gamma=0.99, lam=0.95):
    """rewards [T, B], values [T+1, B] (bootstrap row last), dones [T, B] bool.
    Returns (advantages, returns), each [T, B] float32."""
    lib = _abi.load()
    T, B = rewards.shape
    if tuple(values.shape) != (T + 1, B):
        raise ValueError(f"values must be [T+1, B] = {(T + 1, B)}, got {tuple(values.shape)}")
    if not rewards.is_cuda:
        raise ValueError("rewards must be a GPU tensor (the pass runs on its device)")
    if dones is not None and tuple(dones.shape) != (T, B):
        raise ValueError(f"dones must be [T, B] = {(T, B)}, got {tuple(dones.shape)}")
    # every operand on the rewards' device: a host pointer would fault the kernel
    r = rewards.to(torch.float32).contiguous()
    v = values.to(device=r.device, dtype=torch.float32).contiguous()
    d = dones.to(device=r.device, dtype=torch.uint8).contiguous() if dones is not None else None
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    s = ctypes.c_void_p(torch.cuda.current_stream(r.device).cuda_stream)
    nbytes = lib.pmenv_gae_workspace(T, B)         # horizon split for few envs x long rollouts
    work = torch.empty(max(nbytes // 8, 1), dtype=torch.float64, device=r.device) if nbytes else None
    _abi.check(lib.pmenv_gae_ex(_p(r), _p(v), _p(d), _p(adv), _p(ret), T, B, gamma, lam, _p(work), nbytes, s),
               None, "pmenv_gae_ex")
    return adv, ret


def moments(x):
    """{count, sum, sum of squares} of x in f64 (device tensor [3])."""
    lib = _abi.load()
    if not x.is_cuda:
        raise ValueError("moments needs a GPU tensor")
    x = x.to(torch.float32).contiguous().reshape(-1)
    out = torch.empty(3, dtype=torch.float64, device=x.device)
    work = torch.empty(lib.pmenv_moments_workspace() // 8, dtype=torch.float64, device=x.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    _abi.check(lib.pmenv_moments(_p(x), x.numel(), _p(out), _p(work), s), None, "pmenv_moments")
    return out
