"""A/B of the few-envs GAE horizon split: the product's pmenv_gae_ex (one pass, look-back)
against the tools build's round-3 maps + apply passes (PMENV_GAE=split, read at call time by
the tools build only), in ONE process, interleaved rounds; both checked against the oracle's
recursion on the same inputs (they compose the chunk maps in another order: not bitwise).

    python tools/ab_gae2.py --shapes 4096x512,16384x64,512x64,2048x4096
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pmenv import _abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shapes", default="4096x512,16384x64,512x64,2048x4096,1000x200")
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--calls", type=int, default=50)
ap.add_argument("--variant", default="split", help="the tools build's PMENV_GAE: split | lb16 | lb4x16 | lb16x4")
a = ap.parse_args()
os.environ["PMENV_GAE"] = a.variant
dev = torch.device("cuda:0")
libs = {}
for name, path in (("lookback", os.path.join(ROOT, "pm-rl_amd/pmenv/libpmenv.so")),
                   (a.variant, os.path.join(ROOT, "tools/libpmenv_ab.so"))):
    lib = ctypes.CDLL(path)
    for n, res, args in _abi.SIGNATURES:
        fn = getattr(lib, n, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    libs[name] = lib
P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
out = {}
for shp in a.shapes.split(","):
    T, B = (int(x) for x in shp.split("x"))
    g = torch.Generator(device=dev).manual_seed(T + B)
    r = torch.randn(T, B, device=dev, generator=g)
    v = torch.randn(T + 1, B, device=dev, generator=g)
    d = (torch.rand(T, B, device=dev, generator=g) < 0.003).to(torch.uint8)
    res = {}
    for name, lib in libs.items():
        nb = libs["lookback"].pmenv_gae_workspace(T, B)
        work = torch.empty(max(nb, 8) // 8, dtype=torch.float64, device=dev)
        res[name] = (lib, work, nb, torch.empty_like(r), torch.empty_like(r))

    def call(x):
        lib, work, nb, adv, ret = x
        assert lib.pmenv_gae_ex(P(r), P(v), P(d), P(adv), P(ret), T, B, 0.99, 0.95, P(work), nb, st) == 0
    for x in res.values():
        call(x)
    torch.cuda.synchronize()
    from oracle import gae as or_gae
    oadv, oret = or_gae(r.cpu().numpy(), v.cpu().numpy(), d.cpu().numpy().astype(bool), 0.99, 0.95)
    ok = {}
    for n_, x in res.items():
        ok[n_] = bool(np.allclose(x[3].cpu().numpy(), oadv, rtol=1e-5, atol=1e-5) and
                      np.allclose(x[4].cpu().numpy(), oret, rtol=1e-5, atol=1e-5))
    times = {n_: [] for n_ in res}
    for rd in range(a.rounds):
        for n_ in (list(res) if rd % 2 == 0 else list(reversed(list(res)))):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.calls):
                call(res[n_])
            e1.record()
            torch.cuda.synchronize()
            times[n_].append(e0.elapsed_time(e1) * 1e3 / a.calls)
    alg = T * B * 17 + B * 4
    out[shp] = {n_: {"us": statistics.median(t), "GBs": alg / statistics.median(t) / 1e3, "oracle_ok": ok[n_]}
                for n_, t in times.items()}
    for n_ in res:
        print(f"# gae {shp} {n_:9s} {out[shp][n_]['us']:8.2f} us {out[shp][n_]['GBs']:7.0f} GB/s oracle_ok={ok[n_]}",
              file=sys.stderr, flush=True)
print(json.dumps(out, indent=1))
