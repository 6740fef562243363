"""Advance-step time per shape through the C ABI (raw pmenv_step_ex on prebuilt arguments),
for shapes bench.py does not drive: any F (the market bar has F - 1 channels), windows that
are not 16-B granular, one env. Per shape: the path, us per step (HIP events over K steps,
median of R), env-steps/s and the step's algorithmic HBM bytes (SURVEY.md §8d generalised to
F: read the surviving window N (W-1) F + the bar N (F-1) + the action N floats, write the
window N W F floats, + 20 B of value / reward) against 8 TB/s.

    python tools/bench_shapes.py            # prints one JSON object
"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402

from pmenv import TradingEnv, _abi  # noqa: E402

DEV = torch.device("cuda:0")
K = int(os.environ.get("SHAPES_K", "200"))
R = int(os.environ.get("SHAPES_R", "5"))
PEAK = 8.0e12
# (name, B, N, W, F, in place)
SHAPES = [("config1_1x5x50x5_ip", 1, 5, 50, 5, True), ("config1_1x5x50x5_db", 1, 5, 50, 5, False),
          ("base_1x32x32x8_ip", 1, 32, 32, 8, True), ("feat3_4096x30x50x3_ip", 4096, 30, 50, 3, True), ("feat3_65536x30x50x3_ip", 65536, 30, 50, 3, True),
          ("feat8_4096x30x50x8_ip", 4096, 30, 50, 8, True), ("feat8_65536x30x50x8_ip", 65536, 30, 50, 8, True),
          ("feat8_65536x30x50x8_db", 65536, 30, 50, 8, False), ("odd5_65536x5x50x5_ip", 65536, 5, 50, 5, True)]


def step_bytes(N, W, F):
    return 4 * (N * (W - 1) * F + N * (F - 1) + N + N * W * F) + 20


def main():
    torch.cuda.set_device(DEV)
    lib = _abi.load()
    sel = set(sys.argv[1:])
    out = {"K": K, "R": R}
    for name, B, N, W, F, ip in SHAPES:
        if sel and name not in sel:
            continue
        g = torch.Generator(DEV).manual_seed(B + N + W + F)
        H = 16
        obs = [torch.rand(B, N, W, F, device=DEV, generator=g) + 0.5, torch.empty(B, N, W, F, device=DEV)]
        bars = torch.rand(H, B, N, F - 1, device=DEV, generator=g) + 0.5
        acts = torch.softmax(torch.randn(H, B, N, device=DEV, generator=g), -1)
        env = TradingEnv(num_envs=B, num_assets=N, window=W, features=F, device=DEV, close_channel=min(3, F - 2))
        env.reset(obs[0])
        rew = torch.empty(B, device=DEV)
        sp = ctypes.c_void_p(torch.cuda.current_stream(DEV).cuda_stream)
        args, keep = [], []
        for t in range(H):
            a = _abi.PmenvStepArgs()
            a.action, a.bar, a.reward = acts[t].data_ptr(), bars[t].data_ptr(), rew.data_ptr()
            a.obs = obs[0 if ip else t % 2].data_ptr()
            a.obs_out = None if ip else obs[(t + 1) % 2].data_ptr()
            keep.append(a)
            args.append(ctypes.byref(a))

        def run(k, t0=[0]):
            for _ in range(k):
                assert lib.pmenv_step_ex(env._h, args[t0[0] % H], sp) == 0
                t0[0] += 1
        run(20)
        times = []
        for _ in range(R):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(K)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3 / K)
        us = statistics.median(times)
        by = step_bytes(N, W, F) * B
        parts = env.step_path.split(" | ")         # one name for the non-streaming shapes
        path = parts[-1] if ip else parts[0]
        out[name] = {"path": path, "us_per_step": us, "env_steps_per_s": B / us * 1e6,
                     "bytes_per_step": by, "achieved_GBps": by / us / 1e3, "frac": by / (us * 1e-6) / PEAK}
        print(name, json.dumps(out[name]), file=sys.stderr, flush=True)
        env.close()
        del obs, bars, acts, env
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
