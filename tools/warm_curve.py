"""How long the in-place step takes to reach steady state from a cold process.

Reproduces the driver's bench sequence (synthetic data, env reset, then steps) and
brackets EVERY step's advance launch with HIP events, so the per-step duration of
the first steps is visible. Then idles (as the CPU-baseline leg does) and runs
again. Prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402
from pmenv import TradingEnv, synth, _abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=65536)
ap.add_argument("--steps", type=int, default=600)
ap.add_argument("--idle-s", type=float, default=5.0)
a = ap.parse_args()
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
B, N, W, H = a.envs, 30, 50, 64
lib = _abi.load()
ser = synth.series(H + W, B, N, device=dev)
act = synth.actions(H, B, N, device=dev)
obs = synth.window_from_series(ser, W)
env = TradingEnv(num_envs=B, num_assets=N, window=W, device=dev)
env.reset(obs)
rew = torch.empty(B, device=dev)
stream = torch.cuda.current_stream(dev)
sp = ctypes.c_void_p(stream.cuda_stream)
sa, aa = _abi.PmenvStepArgs(), _abi.PmenvStepArgs()
for x in (sa, aa):
    x.reward, x.obs = rew.data_ptr(), obs.data_ptr()
sa.phases, aa.phases = _abi.PHASE_SCALAR, _abi.PHASE_ADVANCE


def run(steps):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    w0 = torch.cuda.Event(enable_timing=True)
    w0.record(stream)
    for i in range(steps):
        t = i % H
        for x in (sa, aa):
            x.action, x.bar = act[t].data_ptr(), ser[W + t].data_ptr()
        _abi.check(lib.pmenv_step_ex(env._h, ctypes.byref(sa), sp), env._h)
        ev[i][0].record(stream)
        _abi.check(lib.pmenv_step_ex(env._h, ctypes.byref(aa), sp), env._h)
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    us = [x.elapsed_time(y) * 1e3 for x, y in ev]
    return us, w0.elapsed_time(ev[-1][1])


def summary(us):
    out = {"first10": [round(u, 1) for u in us[:10]]}
    for lo, hi in ((0, 5), (5, 25), (25, 50), (50, 100), (100, 200), (200, 400), (400, len(us))):
        if hi <= len(us) and hi > lo:
            out[f"mean_{lo}_{hi}"] = round(statistics.mean(us[lo:hi]), 1)
    return out


cold, cold_ms = run(a.steps)
time.sleep(a.idle_s)
again, again_ms = run(a.steps)
print(json.dumps({"envs": B, "cold": summary(cold), "cold_wall_ms": cold_ms,
                  f"after_{a.idle_s}s_idle": summary(again), "again_wall_ms": again_ms}), flush=True)
