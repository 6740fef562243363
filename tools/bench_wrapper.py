"""Host cost of the Python wrapper: TradingEnv.step (the reference's call shape) against
the raw C ABI call on prebuilt arguments, per step, at small and BASELINE env counts.
Both run the same kernels (AUTO's path); the difference is host work per step, which
only matters where the GPU step is shorter than it."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402
from pmenv import TradingEnv, synth, _abi  # noqa: E402

dev = torch.device("cuda:0")
out = {}
for B in (256, 1024, 4096, 65536):
    N, W, H, steps = 30, 50, 64, 300
    ser = synth.series(W + H, B, N, device=dev)
    act = synth.actions(H, B, N, device=dev)
    obs = synth.window_from_series(ser, W)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=dev)
    env.reset(obs)
    res = {"path": env.step_path.split(" | ")[-1]}
    for mode in ("wrapper", "abi", "wrapper", "abi"):
        lib, sp = _abi.load(), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        rew = torch.empty(B, device=dev)
        prebuilt = []
        for t in range(H):
            a = _abi.PmenvStepArgs()
            a.action, a.bar, a.obs, a.reward = act[t].data_ptr(), ser[W + t].data_ptr(), obs.data_ptr(), rew.data_ptr()
            prebuilt.append((a, ctypes.byref(a)))
        for i in range(20):
            env.step(act[i % H], obs, bar=ser[W + i % H])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if mode == "wrapper":
            for i in range(steps):
                env.step(act[i % H], obs, bar=ser[W + i % H])
        else:
            for i in range(steps):
                lib.pmenv_step_ex(env._h, prebuilt[i % H][1], sp)
        t_host = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        res[mode] = {"us_per_step": t_all / steps * 1e6, "host_us_per_step": t_host / steps * 1e6}
    out[B] = res
    print(B, json.dumps(res), file=sys.stderr, flush=True)
    del env, obs, ser, act
    torch.cuda.empty_cache()
print(json.dumps(out, indent=1))
