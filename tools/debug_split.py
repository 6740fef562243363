"""Debug: step_split_kernel against the two-launch path, per env / window position."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402
from pmenv import TradingEnv, synth  # noqa: E402

DEV = torch.device("cuda:0")
B, N, W, T = int(sys.argv[1]) if len(sys.argv) > 1 else 37, 30, 50, 4
ser = synth.series(W + T, B, N, seed=1, device=DEV)
act = synth.actions(T, B, N, seed=2, device=DEV)
envs = [TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=i) for i in ("split", "two_launch")]
print(envs[0].step_path)
obs = [synth.window_from_series(ser, W) for _ in envs]
for e, o in zip(envs, obs):
    e.reset(o)
for t in range(T):
    lc0 = [e._last_close.clone() for e in envs]
    rs = [e.step(act[t], o, bar=ser[W + t])[0] for e, o in zip(envs, obs)]
    torch.cuda.synchronize()
    y = ser[W + t, 0, :4, 3] / lc0[1].reshape(B, N)[0, :4]
    print("  env0: action", act[t, 0, :4].tolist(), "close", ser[W + t, 0, :4, 3].tolist(),
          "lc split", lc0[0].reshape(B, N)[0, :4].tolist(), "lc two", lc0[1].reshape(B, N)[0, :4].tolist(),
          "y", y.tolist(), "rew", float(rs[0][0]), float(rs[1][0]),
          "lc after", envs[0]._last_close.reshape(B, N)[0, :4].tolist(), envs[1]._last_close.reshape(B, N)[0, :4].tolist(),
          "wnew", envs[0]._w_new.reshape(B, N)[0, :4].tolist(), envs[1]._w_new.reshape(B, N)[0, :4].tolist())
    torch.cuda.synchronize()
    dr = (rs[0] - rs[1]).abs()
    bad = torch.nonzero(dr > 0).flatten().tolist()
    print(f"step {t}: reward envs differing {len(bad)}: {bad[:20]} max {float(dr.max()):.3e}")
    dv = (envs[0].value - envs[1].value).abs()
    print(f"  value envs differing {int((dv > 0).sum())}")
    d = torch.nonzero(obs[0] != obs[1])
    print(f"  window positions differing {d.shape[0]}")
    for row in d[:12].tolist():
        b, n, w, f = row
        print(f"    b{b} n{n} day{w} f{f}: split {float(obs[0][b, n, w, f]):.6f} two {float(obs[1][b, n, w, f]):.6f}")
    if d.shape[0]:
        print("  by feature", torch.bincount(d[:, 3], minlength=5).tolist(), "by day (last 3)",
              [int((d[:, 2] == x).sum()) for x in (W - 3, W - 2, W - 1)])
    dk = (envs[0]._counter != envs[1]._counter).sum()
    dl = (envs[0]._last_close != envs[1]._last_close).sum()
    dw = (envs[0]._w_new != envs[1]._w_new).sum()
    print(f"  counter diffs {int(dk)} last_close diffs {int(dl)} w_new diffs {int(dw)}")
