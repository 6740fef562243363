"""Measure the SURVEY.md §8f kernels (f1 GAE, f2 batched reward, f3 resident-series
advance, f4 replay gather + metrics) against their algorithmic bytes.

Each case is timed with HIP events on torch's current stream (the stream the
wrappers launch on), median of `--reps` calls after warmup. Wrapper overhead
(allocations, ctypes) is inside the timed calls; run under
`rocprofv3 --kernel-trace --stats` for kernel-only durations.
Prints one JSON object; `--out` writes it too.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402

from pmenv import MarketSeries, TradingEnv, rollout, synth, trainer  # noqa: E402
from pmenv.replay import DeviceReplay, trajectory_metrics  # noqa: E402

PEAK_GBS = 8000.0


def timeit(fn, reps, warmup=3):
    st = torch.cuda.current_stream()
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn()
        b.record(st)
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def row(name, us, alg_bytes, **kw):
    gbs = alg_bytes / us / 1e3
    d = {"case": name, "us": round(us, 2), "alg_bytes": int(alg_bytes), "GBs": round(gbs, 1),
         "frac_8TBs": round(gbs / PEAK_GBS, 3)}
    d.update(kw)
    print(json.dumps(d), file=sys.stderr)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    res = []

    # f1: GAE over a time-major rollout, loop (thread per env) vs wave scan
    for T, B, dn in ((256, 65536, True), (2048, 8192, True), (4096, 512, True), (16384, 64, False)):
        r = torch.randn(T, B, device=dev, generator=g)
        v = torch.randn(T + 1, B, device=dev, generator=g)
        d = (torch.rand(T, B, device=dev, generator=g) < 0.01) if dn else None
        alg = T * B * (4 + 4 + 4 + 4 + (1 if dn else 0)) + B * 4
        for mode in ("loop", "scan", "tile", "tile16"):
            os.environ["PMENV_GAE"] = mode.rstrip("16")
            os.environ["PMENV_GAE_U"] = "16" if mode.endswith("16") else "8"
            us = timeit(lambda: rollout.gae(r, v, d, 0.99, 0.95), a.reps)
            res.append(row(f"gae_{mode}", us, alg, T=T, B=B, dones=dn))
        os.environ.pop("PMENV_GAE", None)
        os.environ.pop("PMENV_GAE_U", None)

    # f1: advantage moments (the 24-byte all-reduce's input)
    x = torch.randn(256 * 65536, device=dev, generator=g)
    res.append(row("moments", timeit(lambda: rollout.moments(x), a.reps), x.numel() * 4, n=x.numel()))

    # f2: differentiable batched PG reward, forward + backward
    for B, N in ((65536, 30), (8192, 500)):
        act = torch.randn(B, N, 1, device=dev, generator=g, requires_grad=True)
        vp = torch.rand(B, 1, 1, device=dev, generator=g) + 1.0
        p = 1.0 + 0.01 * torch.randn(B, N, 1, device=dev, generator=g)

        def fwd_bwd():
            act.grad = None
            trainer.pg_reward(act, vp, None, p).backward()
        alg = B * N * 4 * 2 + B * 4 + (B * N * 4 * 2 + B * 4 + B * N * 4)   # fwd reads a, p, v; bwd + grad
        res.append(row("batch_reward_fwd_bwd", timeit(fwd_bwd, a.reps), alg, B=B, N=N))

    # f3: resident series: advance from a per-env day index into one [T, N, 4] series
    B, N, W, T = 65536, 30, 50, 512
    bars = synth.series(T, 1, N, device=dev)[:, 0].contiguous()
    ms = MarketSeries(bars, device=dev)
    starts = ms.random_starts(B, W, 64, generator=torch.Generator().manual_seed(1)).to(dev)
    obs = ms.initial_window(starts, W)
    out = torch.empty_like(obs)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=dev)
    env.reset(obs)
    actn = synth.actions(1, B, N, device=dev)[0]
    day = starts.to(torch.int32) + W
    bufs = [obs, out]
    state = {"i": 0}

    def step_series():
        i = state["i"]
        env.step(actn, bufs[i % 2], series=ms, day=day, out=bufs[(i + 1) % 2])
        day.add_(1)
        state["i"] = i + 1
    res.append(row("step_resident_series", timeit(step_series, a.reps), B * (8 * N * W * 5 + 20),
                   B=B, N=N, W=W))
    del obs, out, bufs, env

    # f4: replay gather (S samples of s, s' windows) and trajectory metrics
    B, N, W, H, S = 4096, 30, 50, 256, 8192
    rb = DeviceReplay(B, N, W, H, ms)
    for h in range(H):
        rb.add(torch.full((B,), W + h, dtype=torch.int32, device=dev), torch.rand(B, N, device=dev),
               torch.randn(B, device=dev))
    h0, e = rb.indices(S, generator=torch.Generator().manual_seed(2))
    alg = S * (2 * N * W * 5 * 4 + N * 4 + 4)          # written windows dominate; reads hit L2
    res.append(row("replay_gather", timeit(lambda: rb.gather(h0, e), a.reps), alg, S=S, N=N, W=W))
    T, B = 252, 65536
    rets = 0.001 * torch.randn(T, B, device=dev, dtype=torch.float64, generator=g)
    vals = torch.cumprod(torch.cat([torch.ones(1, B, device=dev, dtype=torch.float64), 1 + rets]), 0)
    wts = torch.softmax(torch.randn(T + 1, B, 30, device=dev, generator=g), -1)
    alg = T * B * 8 + (T + 1) * B * 8 + (T + 1) * B * 30 * 4 + B * 5 * 8
    res.append(row("trajectory_metrics", timeit(lambda: trajectory_metrics(rets, vals, wts), a.reps), alg,
                   T=T, B=B, N=30))

    doc = {"device": torch.cuda.get_device_name(0), "peak_GBs": PEAK_GBS, "cases": res}
    print(json.dumps(doc, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
