"""Measure the SURVEY.md §8f kernels (f1 GAE + moments, f2 batched reward, f3
resident-series advance, f4 replay gather + metrics) against their algorithmic bytes.

Every case calls the C ABI directly on preallocated device buffers (what a training
loop does), timed with HIP events on torch's current stream — the stream the calls
enqueue on — per call, as the median over `--reps` groups of 10 back-to-back calls
after warmup. A case is one ABI call (its kernels and the boundaries between them,
no allocation). Run under
`rocprofv3 --kernel-trace --stats` for per-kernel durations.
Prints one JSON object; `--out` writes it too.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PMENV_LIB", os.path.join(ROOT, "tools", "libpmenv_ab.so"))  # the A/B knobs: tools build
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402

from pmenv import MarketSeries, TradingEnv, synth, _abi  # noqa: E402
from pmenv.replay import DeviceReplay  # noqa: E402

PEAK_GBS = 8000.0


def P(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def timeit(fn, reps, warmup=3, inner=10):
    """Median over `reps` groups of `inner` back-to-back calls (per call): launch
    latency overlaps the previous call, as in a training loop."""
    st = torch.cuda.current_stream()
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(inner):
            fn()
        b.record(st)
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / inner)
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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="")
    ap.add_argument("--only", default="", help="comma list of f1,f2,f3,f4 (default: all)")
    a = ap.parse_args()
    only = set(a.only.split(",")) if a.only else {"f1", "f2", "f3", "f4"}
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lib = _abi.load()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device=dev).manual_seed(0)
    res = []

    def ck(rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed: {rc}")

    if "f1" in only:
        # GAE over a time-major rollout: per-env loop, wave scan, tiled scan (U = 8, 16)
        for T, B, dn in ((256, 65536, True), (256, 16384, True), (256, 4096, True), (2048, 8192, True),
                         (4096, 512, True), (16384, 64, False)):
            r = torch.randn(T, B, device=dev, generator=g)
            v = torch.randn(T + 1, B, device=dev, generator=g)
            d = (torch.rand(T, B, device=dev, generator=g) < 0.01).to(torch.uint8) if dn else None
            adv, ret = torch.empty_like(r), torch.empty_like(r)
            alg = T * B * (4 + 4 + 4 + 4 + (1 if dn else 0)) + B * 4
            big = T * B <= (1 << 24)
            modes = {"loop": {"PMENV_GAE": "loop"}, "scan": {"PMENV_GAE": "scan"}} if big else {}
            modes.update({"tile": {"PMENV_GAE": "tile", "PMENV_GAE_U": "8"},
                          "tile16": {"PMENV_GAE": "tile", "PMENV_GAE_U": "16"},
                          "tile_occ8": {"PMENV_GAE": "tile8"},
                          "stream8": {"PMENV_GAE": "stream", "PMENV_GAE_P": "8"},
                          "stream16": {"PMENV_GAE": "stream", "PMENV_GAE_P": "16"},
                          "stream32": {"PMENV_GAE": "stream", "PMENV_GAE_P": "32"},
                          "tile_nt": {"PMENV_GAE_SP": "2"},
                          "tile_sc1": {"PMENV_GAE_SP": "16"},
                          "auto": {}})
            nbytes = lib.pmenv_gae_workspace(T, B)
            work = torch.empty(max(nbytes // 8, 1), dtype=torch.float64, device=dev)
            gk = ("PMENV_GAE", "PMENV_GAE_U", "PMENV_GAE_P", "PMENV_GAE_SP")
            outs = {}
            for mode, env in modes.items():
                for k in gk:
                    os.environ.pop(k, None)
                os.environ.update(env)
                # auto = what rollout.gae runs: pmenv_gae_ex with its workspace (horizon split)
                call = lambda: ck(lib.pmenv_gae_ex(P(r), P(v), P(d), P(adv), P(ret), T, B, 0.99, 0.95,  # noqa: E731
                                                   P(work), nbytes, st), "gae")
                call()
                outs[mode] = (adv.clone(), ret.clone())
                us = timeit(call, a.reps)
                same_tile = bool(torch.equal(outs[mode][0], outs["tile"][0])) if "tile" in outs else None
                same_loop = bool(torch.equal(outs[mode][0], outs["loop"][0])) if "loop" in outs else None
                err = float((outs[mode][0] - outs["tile"][0]).abs().max()) if "tile" in outs else None
                res.append(row(f"gae_{mode}", us, alg, T=T, B=B, dones=dn, split=bool(nbytes) and mode == "auto",
                               same_bits_tile=same_tile, same_bits_loop=same_loop, max_abs_vs_tile=err))
            del outs
            for k in gk:
                os.environ.pop(k, None)
            del r, v, d, adv, ret
        # compact on-policy rollout: minibatch windows re-materialised from the resident
        # series + recorded w' (pmenv_rollout_gather), config 2's shape (4,096 envs x 32 steps)
        for Bc, Tr, S in ((4096, 32, 4096), (4096, 32, 32768), (65536, 64, 8192)):
            N_, W_ = 30, 50
            Ts = Tr + W_ + 8
            ser_c = torch.rand(Ts, N_, 4, device=dev, generator=g)
            start = torch.randint(0, 8, (Bc,), device=dev, generator=g).to(torch.int32)
            wts = torch.rand(Tr, Bc, N_, device=dev, generator=g)
            tix = torch.randint(0, Tr + 1, (S,), device=dev, generator=g).to(torch.int32)
            eix = torch.randint(0, Bc, (S,), device=dev, generator=g).to(torch.int32)
            out_c = torch.empty(S, N_, W_, 5, device=dev)
            call = lambda: ck(lib.pmenv_rollout_gather(P(ser_c), Ts, N_, 5, W_, P(start), P(wts), Tr, Bc, 0,  # noqa: E731
                                                       P(tix), P(eix), S, P(out_c), st), "rollout_gather")
            outs = {}
            # the product's LDS-staged tile, the wave-per-row and float-per-thread forms (tools)
            forms = (("tile", None), ("rows", "PMENV_RGATHER_ROWS"), ("elem", "PMENV_RGATHER_ELEM"),
                     ("tile_nt", "PMENV_RGATHER_NT=2"), ("tile_sc1", "PMENV_RGATHER_NT=16"),
                     ("tile_nt_sc1", "PMENV_RGATHER_NT=18"))
            for form, knob in forms:
                for k in ("PMENV_RGATHER_ELEM", "PMENV_RGATHER_ROWS", "PMENV_RGATHER_NT"):
                    os.environ.pop(k, None)
                if knob:
                    k, _, val = knob.partition("=")
                    os.environ[k] = val or "1"
                call()
                outs[form] = out_c.clone()
                res.append(row(f"rollout_gather_{form}", timeit(call, a.reps), S * N_ * W_ * 5 * 4, B=Bc, T=Tr, S=S,
                               N=N_, W=W_, same_bits=bool(torch.equal(outs[form], outs["tile"]))))
            for k in ("PMENV_RGATHER_ELEM", "PMENV_RGATHER_ROWS", "PMENV_RGATHER_NT"):
                os.environ.pop(k, None)
            del outs
            del ser_c, wts, out_c
        # advantage moments (the 24-byte all-reduce's input)
        for n in (256 * 65536, 256 * 4096):
            x = torch.randn(n, device=dev, generator=g)
            out = torch.empty(3, dtype=torch.float64, device=dev)
            work = torch.empty(lib.pmenv_moments_workspace() // 8, dtype=torch.float64, device=dev)
            us = timeit(lambda: ck(lib.pmenv_moments(P(x), n, P(out), P(work), st), "moments"), a.reps)
            res.append(row("moments", us, n * 4, n=n))

    if "f2" in only:
        # differentiable batched PG reward: forward (reward only; the product's two launches
        # and the tools build's one-launch forms under PMENV_BR_ONE, interleaved) and backward
        for B, N in ((65536, 30), (16384, 30), (4096, 30), (8192, 500)):
            act = torch.randn(B, N, device=dev, generator=g)
            vp = torch.rand(B, device=dev, generator=g) + 1.0
            p = 1.0 + 0.01 * torch.randn(B, N, device=dev, generator=g)
            work = torch.empty(lib.pmenv_batch_reward_workspace(B) // 8, dtype=torch.float64, device=dev)
            rout = torch.empty((), device=dev)
            go = torch.ones((), device=dev)
            ga = torch.empty_like(act)
            fwd = lambda: ck(lib.pmenv_batch_reward_forward(P(act), P(vp), P(p), B, N, 0, 0, 1.0, P(work),  # noqa: E731
                                                            P(rout), None, st), "fwd")
            bwd = lambda: ck(lib.pmenv_batch_reward_backward(P(act), P(vp), P(p), B, N, 0, 1.0, P(work), P(go),  # noqa: E731
                                                             P(ga), st), "bwd")
            f_bytes = B * N * 4 * 2 + B * 4
            forms = {"two": {}, "one": {"PMENV_BR_ONE": "1"}, "one_fence_all": {"PMENV_BR_ONE": "1", "PMENV_BR_FENCE": "0"},
                     "one_grid256": {"PMENV_BR_ONE": "1", "PMENV_BR_GRID": "256"},
                     "one_grid512": {"PMENV_BR_ONE": "1", "PMENV_BR_GRID": "512"}}
            knobs = ("PMENV_BR_ONE", "PMENV_BR_FENCE", "PMENV_BR_GRID")

            def use(form):
                for k in knobs:
                    os.environ.pop(k, None)
                os.environ.update(forms[form])
            outs = {}
            for form in forms:                          # the same bits every way
                use(form)
                fwd()
                outs[form] = (rout.clone(), work[6 * B:6 * B + 5].clone())
            same = all(torch.equal(outs[f][0], outs["two"][0]) and torch.equal(outs[f][1], outs["two"][1])
                       for f in forms)
            ts = {f: [] for f in forms}
            for _ in range(3):
                for form in forms:
                    use(form)
                    ts[form].append(timeit(fwd, a.reps))
            use("two")
            for form in forms:
                res.append(row(f"batch_reward_fwd_{form}", statistics.median(ts[form]), f_bytes, B=B, N=N,
                               same_bits=same))
            res.append(row("batch_reward_bwd", timeit(bwd, a.reps), f_bytes + B * N * 4, B=B, N=N))

    if "f3" in only or "f4" in only:
        B, N, W, T = 65536, 30, 50, 512
        bars = synth.series(T, 1, N, device=dev)[:, 0].contiguous()
        ms = MarketSeries(bars, device=dev)
    if "f3" in only:
        # resident series: the env step with a per-env day index into one [T, N, 4] series
        starts = ms.random_starts(B, W, 64, generator=torch.Generator().manual_seed(1)).to(dev)
        obs = ms.initial_window(starts, W)
        out = torch.empty_like(obs)
        env = TradingEnv(num_envs=B, num_assets=N, window=W, device=dev)
        env.reset(obs)
        actn = synth.actions(1, B, N, device=dev)[0]
        day = starts.to(torch.int32) + W
        rew = torch.empty(B, device=dev)
        bufs = [obs, out]
        state = {"i": 0}
        args = _abi.PmenvStepArgs()
        args.action, args.bar, args.reward = actn.data_ptr(), ms.bars.data_ptr(), rew.data_ptr()
        args.day, args.series_days = day.data_ptr(), T

        def step_series(db):
            i = state["i"]
            args.obs = bufs[i % 2].data_ptr()
            args.obs_out = bufs[(i + 1) % 2].data_ptr() if db else None
            ck(lib.pmenv_step_ex(env._h, ctypes.byref(args), st), "step")
            if db:
                state["i"] = i + 1
        for db in (True, False):
            us = timeit(lambda: step_series(db), a.reps)
            res.append(row("step_resident_series", us, B * (8 * N * W * 5 + 20), B=B, N=N, W=W,
                           windows="double" if db else "inplace"))
        del obs, out, bufs, env
    if "f4" in only:
        # replay gather (S samples of s, s' windows) and trajectory metrics
        B, N, W, H, S = 4096, 30, 50, 256, 8192
        rb = DeviceReplay(B, N, W, H, ms)
        for h in range(H):
            rb.add(torch.full((B,), W + h, dtype=torch.int32, device=dev), torch.rand(B, N, device=dev),
                   torch.randn(B, device=dev))
        h0, e = rb.indices(S, generator=torch.Generator().manual_seed(2))
        s_ = torch.empty(S, N, W, 5, device=dev)
        s2 = torch.empty_like(s_)
        ao = torch.empty(S, N, device=dev)
        ro = torch.empty(S, device=dev)
        sb = ms.bars

        def gather():
            ck(lib.pmenv_replay_gather(P(sb), sb.shape[0], N, 5, W, P(rb.days), P(rb.actions), P(rb.rewards), H, B,
                                       P(h0), P(e), S, P(s_), P(s2), P(ao), P(ro), st), "gather")
        alg = S * (2 * N * W * 5 * 4 + N * 4 + 4)          # written windows dominate; reads hit L2
        for mode in ("f5", "lds"):
            os.environ.pop("PMENV_REPLAY_LDS", None)
            if mode == "lds":
                os.environ["PMENV_REPLAY_LDS"] = "1"
            res.append(row(f"replay_gather_{mode}", timeit(gather, a.reps), alg, S=S, N=N, W=W))
        os.environ.pop("PMENV_REPLAY_LDS", None)
        del rb, s_, s2
        for T, B in ((252, 65536), (252, 4096)):
            rets = 0.001 * torch.randn(T, B, device=dev, dtype=torch.float64, generator=g)
            vals = torch.cumprod(torch.cat([torch.ones(1, B, device=dev, dtype=torch.float64), 1 + rets]), 0)
            wts = torch.softmax(torch.randn(T + 1, B, 30, device=dev, generator=g), -1)
            out = torch.empty(B, 5, dtype=torch.float64, device=dev)
            alg = T * B * 8 + (T + 1) * B * 8 + (T + 1) * B * 30 * 4 + B * 5 * 8
            for mode in ("fused", "seg", "walk"):
                os.environ.pop("PMENV_METRICS_WALK", None)
                os.environ.pop("PMENV_METRICS_FUSED", None)
                if mode == "walk":
                    os.environ["PMENV_METRICS_WALK"] = "1"
                if mode == "seg":                       # the two passes as two launches
                    os.environ["PMENV_METRICS_FUSED"] = "0"
                us = timeit(lambda: ck(lib.pmenv_metrics(P(rets), P(vals), P(wts), T, B, 30, 0.04, 252.0, P(out), st),
                                       "metrics"), a.reps)
                res.append(row(f"trajectory_metrics_{mode}", us, alg, T=T, B=B, N=30))
            os.environ.pop("PMENV_METRICS_WALK", None)
            os.environ.pop("PMENV_METRICS_FUSED", None)

    doc = {"device": torch.cuda.get_device_name(0), "peak_GBs": PEAK_GBS, "cases": res}
    print(json.dumps(doc, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
