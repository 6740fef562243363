"""The flat one-launch step per step at 65,536 x 30: host-sequenced (the default until a
step is captured), device-sequenced eager (flat_seq_kernel + step_flat_kernel, after a
capture) and device-sequenced replayed from a hipGraph of 16 steps, against the
two-launch path; interleaved rounds, one process."""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402
from pmenv import TradingEnv, synth, _abi  # noqa: E402

dev = torch.device("cuda:0")
B, N, W, H, S = 65536, 30, 50, 32, 16
ser = synth.series(W + H, B, N, device=dev)
act = synth.actions(H, B, N, device=dev)
lib = _abi.load()
envs = {}
for name, impl in (("two_launch", "two_launch"), ("flat_host", "flat"), ("flat_device", "flat"),
                   ("flat_graph", "flat")):
    obs = synth.window_from_series(ser, W)
    e = TradingEnv(num_envs=B, num_assets=N, window=W, device=dev, step_impl=impl)
    e.reset(obs)
    envs[name] = (e, obs, torch.empty(B, device=dev))
graphs = {}
for name in ("flat_device", "flat_graph"):
    e, obs, rew = envs[name]
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for t in range(S):
            lib.pmenv_step(e._h, ctypes.c_void_p(act[t].data_ptr()), None, ctypes.c_void_p(ser[W + t].data_ptr()),
                           ctypes.c_void_p(obs.data_ptr()), ctypes.c_void_p(rew.data_ptr()), s)
    graphs[name] = g
    assert "device-sequenced" in e.step_path
stream = torch.cuda.current_stream()
sp = ctypes.c_void_p(stream.cuda_stream)
times = {k: [] for k in envs}
for r in range(8):
    for name, (e, obs, rew) in envs.items():
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(stream)
        if name == "flat_graph":
            graphs[name].replay()
        else:
            for t in range(S):
                lib.pmenv_step(e._h, ctypes.c_void_p(act[t].data_ptr()), None, ctypes.c_void_p(ser[W + t].data_ptr()),
                               ctypes.c_void_p(obs.data_ptr()), ctypes.c_void_p(rew.data_ptr()), sp)
        b.record(stream)
        torch.cuda.synchronize()
        if r > 0:
            times[name].append(a.elapsed_time(b) * 1e3 / S)
out = {k: {"median_us": statistics.median(v), "min_us": min(v)} for k, v in times.items()}
ref = envs["two_launch"][1]
for k in ("flat_host", "flat_device", "flat_graph"):
    out[k]["window_equals_two_launch"] = bool(torch.equal(envs[k][1], ref))
print(json.dumps(out, indent=1))
