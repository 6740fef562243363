"""The reference's surface contract (trading_env.py:44-105: the caller hands each day's window
and the price relatives, the env rewrites channel F-1 from its ring) with device tensors at
vectorised sizes, through the raw C ABI (pmenv_step_ex, bar = NULL): us per step (HIP events
over K steps, median of R) and the step's bytes — read the action, prices and the ring rows
(N (W + 2) floats), write channel F-1 (N W floats, every F-th float of the window) and 20 B of
state / reward per env — against 8 TB/s.

    python tools/bench_surface.py       # prints one JSON object
    SURF_LIBS=pm-rl_amd/pmenv/libpmenv.so,tools/libpmenv_ab.so PMENV_SURF_CHUNK=0 python tools/bench_surface.py
                                        # two builds interleaved in one process, bits compared
"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402

from pmenv import _abi  # noqa: E402

DEV = torch.device("cuda:0")
K = int(os.environ.get("SURF_K", "50"))
R = int(os.environ.get("SURF_R", "5"))
SHAPES = [(1, 5, 50, 5), (4096, 30, 50, 5), (16384, 30, 50, 5), (65536, 30, 50, 5), (16384, 30, 50, 8)]
if os.environ.get("SURF_SHAPES"):                  # e.g. SURF_SHAPES=65536x30x50x5 (profiling passes)
    SHAPES = [tuple(int(x) for x in s.split("x")) for s in os.environ["SURF_SHAPES"].split(",")]


def load(path):
    lib = ctypes.CDLL(path)
    for name, res, argt in _abi.SIGNATURES:
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, argt
    return lib


class Env:
    def __init__(self, lib, B, N, W, F):
        self.lib = lib
        c = _abi.PmenvCfg()
        lib.pmenv_cfg_default(ctypes.byref(c), B, N, W, F)
        c.close_channel = min(3, F - 2)
        self.h = ctypes.c_void_p()
        assert lib.pmenv_create(ctypes.byref(c), 0, ctypes.byref(self.h)) == 0
        g = torch.Generator(DEV).manual_seed(B)
        self.obs = torch.rand(B, N, W, F, device=DEV, generator=g) + 0.5
        self.H = 8
        self.prices = torch.rand(self.H, B, N, device=DEV, generator=g) * 0.1 + 0.95
        self.acts = torch.softmax(torch.randn(self.H, B, N, device=DEV, generator=g), -1)
        self.rew = torch.empty(B, device=DEV)
        sp = ctypes.c_void_p(torch.cuda.current_stream(DEV).cuda_stream)
        assert lib.pmenv_reset(self.h, ctypes.c_void_p(self.obs.data_ptr()), None, sp) == 0
        self.args = []
        for t in range(self.H):
            a = _abi.PmenvStepArgs()
            a.action, a.prices, a.obs, a.reward = (self.acts[t].data_ptr(), self.prices[t].data_ptr(),
                                                   self.obs.data_ptr(), self.rew.data_ptr())
            self.args.append(a)
        self.t = 0

    def run(self, k):
        sp = ctypes.c_void_p(torch.cuda.current_stream(DEV).cuda_stream)
        for _ in range(k):
            assert self.lib.pmenv_step_ex(self.h, ctypes.byref(self.args[self.t % self.H]), sp) == 0
            self.t += 1

    def close(self):
        torch.cuda.synchronize()
        self.lib.pmenv_destroy(self.h)


def timed(env):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    env.run(K)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / K


def main():
    torch.cuda.set_device(DEV)
    paths = os.environ.get("SURF_LIBS", "").split(",") if os.environ.get("SURF_LIBS") else [None]
    libs = {(p or "product"): (load(os.path.join(ROOT, p)) if p else _abi.load()) for p in paths}
    out = {"K": K, "R": R}
    for B, N, W, F in SHAPES:
        envs = {n: Env(lib, B, N, W, F) for n, lib in libs.items()}
        for e in envs.values():
            e.run(10)
        times = {n: [] for n in envs}
        for _ in range(R):
            for n, e in envs.items():
                times[n].append(timed(e))
        by = B * (4 * (N * (W + 2) + N * W) + 20)
        o = {}
        for n in envs:
            us = statistics.median(times[n])
            o[n] = {"us_per_step": us, "env_steps_per_s": B / us * 1e6, "frac": by / (us * 1e-6) / 8e12}
        o["bytes_per_step"] = by
        if len(envs) == 2:
            a, b = list(envs.values())
            o["windows_equal"] = bool(torch.equal(a.obs.view(torch.int32), b.obs.view(torch.int32)))
            o["rewards_equal"] = bool(torch.equal(a.rew.view(torch.int32), b.rew.view(torch.int32)))
        out[f"{B}x{N}x{W}x{F}"] = o
        print(f"{B}x{N}x{W}x{F}", json.dumps(o), file=sys.stderr, flush=True)
        for e in envs.values():
            e.close()
        del envs
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
