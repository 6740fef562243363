"""One train/on_policy.py iteration (rollout -> update -> returns) at BASELINE config 2
(4,096 envs x 30 assets, A2C on-policy, 1 GPU) over pmenv.on_policy.OnPolicy, with
the time split between the env step, the policy and the update.

The policy is the small WindowPolicy stand-in (the reference's LSRE-CANN is out of
scope), so the policy share below is a floor, not the reference's network cost.
Prints one JSON object; `--out` writes it too.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402

from pmenv import TradingEnv, synth  # noqa: E402
from pmenv.on_policy import OnPolicy, WindowPolicy  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=4096)
ap.add_argument("--assets", type=int, default=30)
ap.add_argument("--window", type=int, default=50)
ap.add_argument("--horizon", type=int, default=32)
ap.add_argument("--batch-size", type=int, default=4096)
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--out", default="")
a = ap.parse_args()
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
B, N, W, T = a.envs, a.assets, a.window, a.horizon
ser = synth.series(W + T, B, N, device=dev)                      # [W+T, B, N, 4]
obs0 = synth.window_from_series(ser, W)
bars = [ser[W + t] for t in range(T)]
env = TradingEnv(num_envs=B, num_assets=N, window=W, device=dev)
torch.manual_seed(0)
loop = OnPolicy(env, WindowPolicy(W).to(dev), horizon=T, batch_size=a.batch_size,
                generator=torch.Generator().manual_seed(1))
st = torch.cuda.current_stream()
E = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

# env-step events: wrap TradingEnv.step for the rollout (same launches, timed)
step_ms = []
_step = env.step


def timed_step(*args, **kw):
    e0, e1 = E(), E()
    e0.record(st)
    out = _step(*args, **kw)
    e1.record(st)
    step_ms.append((e0, e1))
    return out


env.step = timed_step
vals = torch.randn(T + 1, B, device=dev)                       # critic values (timing only)
res = []
for it in range(a.iters + 1):
    step_ms.clear()
    t0, t1, t2, t3 = E(), E(), E(), E()
    t0.record(st)
    rewards = loop.rollout(obs0, bars)
    t1.record(st)
    losses = loop.update()
    t2.record(st)
    adv, ret = loop.buf.returns(vals)
    t3.record(st)
    torch.cuda.synchronize()
    if it == 0:
        continue                                            # warmup (allocator, kernels)
    env_ms = sum(x.elapsed_time(y) for x, y in step_ms)
    roll_ms = t0.elapsed_time(t1)
    res.append({"rollout_ms": roll_ms, "env_step_ms": env_ms, "policy_and_buffer_ms": roll_ms - env_ms,
                "update_ms": t1.elapsed_time(t2), "returns_ms": t2.elapsed_time(t3),
                "updates": int(losses.numel())})
med = {k: sorted(r[k] for r in res)[len(res) // 2] for k in res[0]}
iter_ms = med["rollout_ms"] + med["update_ms"] + med["returns_ms"]
doc = {"device": torch.cuda.get_device_name(0), "envs": B, "assets": N, "window": W, "horizon": T,
       "batch_size": a.batch_size, "median": med,
       "env_steps_per_s_rollout": B * T / (med["rollout_ms"] / 1e3),
       "env_steps_per_s_env_only": B * T / (med["env_step_ms"] / 1e3),
       "env_steps_per_s_iteration": B * T / (iter_ms / 1e3),
       "env_share_of_iteration": med["env_step_ms"] / iter_ms,
       "note": "policy = WindowPolicy stand-in (per-asset MLP), update = A2C._loss via the fused HIP op"}
print(json.dumps(doc, indent=1))
if a.out:
    with open(a.out, "w") as f:
        json.dump(doc, f, indent=1)
