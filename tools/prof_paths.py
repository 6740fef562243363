"""Run a few step paths / modes back to back (for rocprofv3 --kernel-trace): each config
steps its own handle `--steps` times after a warm-up. Kernel times come from the trace."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402
from pmenv import TradingEnv, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=65536)
ap.add_argument("--assets", type=int, default=30)
ap.add_argument("--steps", type=int, default=30)
ap.add_argument("--configs", default="two_launch:0,two_launch:0.0025,flat:0,flat:0.0025")
a = ap.parse_args()
dev = torch.device("cuda:0")
B, N, W, H = a.envs, a.assets, 50, 16
ser = synth.series(W + H, B, N, device=dev)
act = synth.actions(H, B, N, device=dev)
for spec in a.configs.split(","):
    impl, comm = spec.split(":")
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=dev, step_impl=impl, commission=float(comm))
    obs = synth.window_from_series(ser, W)
    env.reset(obs)
    for t in range(a.steps + 5):
        env.step(act[t % H], obs, bar=ser[W + t % H])
    torch.cuda.synchronize()
    print(spec, env.step_path, flush=True)
    del env, obs
    torch.cuda.empty_cache()
