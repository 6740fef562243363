"""Do the steps right after a reset run slower than steps deep into a run?

bench.py's sequence is: a 64-step parity leg, then the window re-initialised and the
env reset, W warm-up steps and the K timed steps. This times, in one process and in
alternating rounds, K steps that follow (a) that reset, and (b) the same 64 + W steps
with no reset in between — every step bracketed by HIP events. Prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402
from pmenv import TradingEnv, synth, _abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=65536)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--lead", type=int, default=64)
ap.add_argument("--rounds", type=int, default=6)
a = ap.parse_args()
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
B, N, W, H = a.envs, 30, 50, 256
lib = _abi.load()
ser = synth.series(H + W, B, N, device=dev)
act = synth.actions(H, B, N, device=dev)
obs = synth.window_from_series(ser, W)
env = TradingEnv(num_envs=B, num_assets=N, window=W, device=dev)
rew = torch.empty(B, device=dev)
stream = torch.cuda.current_stream(dev)
sp = ctypes.c_void_p(stream.cuda_stream)
args = _abi.PmenvStepArgs()
args.reward, args.obs = rew.data_ptr(), obs.data_ptr()
day = [0]


def steps(n, ev=None):
    for i in range(n):
        t = day[0] % H
        day[0] += 1
        args.action, args.bar = act[t].data_ptr(), ser[W + t].data_ptr()
        if ev is not None:
            ev[i][0].record(stream)
        _abi.check(lib.pmenv_step_ex(env._h, ctypes.byref(args), sp), env._h)
        if ev is not None:
            ev[i][1].record(stream)


def leg(reset):
    obs.copy_(synth.window_from_series(ser, W))
    env.reset(obs)
    day[0] = 0
    steps(a.lead)
    if reset:
        obs.copy_(synth.window_from_series(ser, W))
        env.reset(obs)
        day[0] = 0
    steps(a.warmup)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    steps(a.steps, ev)
    torch.cuda.synchronize()
    return [x.elapsed_time(y) * 1e3 for x, y in ev]


res = {"after_reset": [], "continued": []}
for r in range(a.rounds):
    for name, rs in (("after_reset", True), ("continued", False)):
        res[name].append(leg(rs))
out = {"envs": B, "steps": a.steps, "warmup": a.warmup, "lead": a.lead, "path": env.step_path}
for name, runs in res.items():
    flat = [u for run in runs[1:] for u in run]
    out[name] = {"median_us": round(statistics.median(flat), 1), "mean_us": round(statistics.mean(flat), 1),
                 "first5_mean_us": round(statistics.mean([u for run in runs[1:] for u in run[:5]]), 1),
                 "last5_mean_us": round(statistics.mean([u for run in runs[1:] for u in run[-5:]]), 1)}
print(json.dumps(out), flush=True)
