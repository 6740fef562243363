"""Launch-bound small batches: the fused env step launched eagerly from Python (one
pmenv_step call per step) against the same T steps captured once into a hipGraph
(torch.cuda.CUDAGraph over the C ABI calls) and replayed. Per-step wall time and
env-steps/s per batch size; both runs must produce the same rewards and windows.

    python tools/bench_graph.py [--envs 64,256,1024,4096] [--steps 64]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402

from pmenv import TradingEnv, synth, _abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", default="64,256,1024,4096")
ap.add_argument("--assets", type=int, default=30)
ap.add_argument("--window", type=int, default=50)
ap.add_argument("--steps", type=int, default=64)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--out", default="")
a = ap.parse_args()
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
lib = _abi.load()
N, W, T = a.assets, a.window, a.steps
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
res = []
for B in (int(x) for x in a.envs.split(",")):
    ser = synth.series(W + T, B, N, device=dev)
    act = synth.actions(T, B, N, device=dev)
    obs0 = synth.window_from_series(ser, W)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=dev)
    obs = obs0.clone()
    rew = torch.empty(T, B, device=dev)
    st = torch.cuda.current_stream()

    def run_eager():
        s = ctypes.c_void_p(st.cuda_stream)
        for t in range(T):
            lib.pmenv_step(env._h, P(act[t]), None, P(ser[W + t]), P(obs), P(rew[t]), s)

    def reset():
        obs.copy_(obs0)
        env.reset(obs)

    # eager: host-launched steps
    reset()
    run_eager()
    torch.cuda.synchronize()
    eager = []
    for _ in range(a.reps):
        reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run_eager()
        torch.cuda.synchronize()
        eager.append(time.perf_counter() - t0)
    r_eager, o_eager = rew.clone(), obs.clone()
    # graph: the T steps captured once, replayed
    reset()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for t in range(T):
            _abi.check(lib.pmenv_step(env._h, P(act[t]), None, P(ser[W + t]), P(obs), P(rew[t]), s), env._h)
    graph = []
    for _ in range(a.reps):
        reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        graph.append(time.perf_counter() - t0)
    same = bool(torch.equal(rew, r_eager) and torch.equal(obs, o_eager))
    e_us, g_us = sorted(eager)[len(eager) // 2] / T * 1e6, sorted(graph)[len(graph) // 2] / T * 1e6
    d = {"envs": B, "eager_us_per_step": round(e_us, 2), "graph_us_per_step": round(g_us, 2),
         "eager_env_steps_per_s": B / e_us * 1e6, "graph_env_steps_per_s": B / g_us * 1e6,
         "speedup": round(e_us / g_us, 2), "identical": same, "step_path": env.step_path.split(" |")[0]}
    print(json.dumps(d), file=sys.stderr)
    res.append(d)
    del g
doc = {"device": torch.cuda.get_device_name(0), "assets": N, "window": W, "steps_per_graph": T, "cases": res}
print(json.dumps(doc, indent=1))
if a.out:
    with open(a.out, "w") as f:
        json.dump(doc, f, indent=1)
