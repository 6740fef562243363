"""Bit fingerprints of the env step (trading_env.py:54-105 on every step path AUTO picks and
the paths it can be forced to), the way tools/f2_bits.py fingerprints the batched reward:
windows, rewards and state after a few steps, with raw actions (the softmax branch, so the
f64 exp runs) and simplex actions, at every scalar-step form (N = 8 / 16 packed, 30 / 64
register, 100 / 300 / 500 packed strided) and reward kind. A library rebuilt with code that
must not move a bit (e.g. fmath.h's exp_f64) is checked against another build:

    python tools/step_bits.py --lib tools/libpmenv_old.so > old.json
    python tools/step_bits.py --check old.json
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))

CASES = [(512, 8), (512, 16), (1024, 30), (256, 64), (128, 100), (64, 300), (64, 500)]
KINDS = ["log_returns", "returns", "sharpe_ratio", "diff_sharpe"]
PATHS = ["auto", "one_launch", "two_launch", "flat", "relay"]


def fingerprints(dev="cuda:0"):
    import torch
    from pmenv import TradingEnv, synth
    out = {}
    W, T = 20, 6
    for B, N in CASES:
        ser = synth.series(W + T, B, N, seed=B + N, device=dev)
        raw = synth.actions(T, B, N, seed=N, device=dev)
        g = torch.Generator(device=dev).manual_seed(N)
        gauss = torch.randn(T, B, N, device=dev, generator=g)
        for kind in KINDS:
            for path in PATHS:
                try:
                    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=dev, reward=kind,
                                     commission=0.0025 if kind == "returns" else 0.0, step_impl=path)
                except Exception as e:                   # a path the shape does not support
                    out[f"{B}x{N}/{kind}/{path}"] = f"n/a: {type(e).__name__}"
                    continue
                obs = synth.window_from_series(ser, W)
                env.reset(obs)
                h = hashlib.sha256()
                for t in range(T):
                    a = gauss[t] if t % 2 else raw[t]      # raw Gaussian scores: softmax; simplex: none
                    r, _ = env.step(a, obs, bar=ser[W + t])
                    h.update(r.cpu().numpy().tobytes())
                h.update(obs.cpu().numpy().tobytes())
                h.update(env.value.cpu().numpy().tobytes())
                out[f"{B}x{N}/{kind}/{path}"] = h.hexdigest()[:32]
                del env, obs
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", help="load this libpmenv build instead of the in-tree one")
    ap.add_argument("--check", help="compare against these fingerprints instead of printing")
    a = ap.parse_args()
    if a.lib:
        from pmenv import _abi
        _abi.LIB_PATH = os.path.abspath(a.lib)
    got = fingerprints()
    if not a.check:
        print(json.dumps(got, indent=1, sort_keys=True))
        sys.exit(0)
    want = json.load(open(a.check))
    bad = sorted(k for k in want if got.get(k) != want[k])
    print(f"step_bits: {len(want) - len(bad)} of {len(want)} fingerprints equal" + (f"; moved: {bad[:8]}" if bad else ""))
    sys.exit(1 if bad or set(got) != set(want) else 0)
