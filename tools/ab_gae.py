"""A/B the GAE kernels (env knobs read at each call) in ONE process, interleaved
rounds. Variants are '+'-joined KEY=VALUE knob sets; variants with the same
segment length (PMENV_GAE_NW x PMENV_GAE_U) must agree bit for bit, all of them within 1e-5 of
the first.

    python tools/ab_gae.py --shapes 256x65536,256x16384 \
        --variants "PMENV_GAE=tile+PMENV_GAE_U=8,PMENV_GAE=tile+PMENV_GAE_U=8+PMENV_GAE_E=2"
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
from pmenv import _abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shapes", default="256x65536,256x16384,256x4096")
ap.add_argument("--variants", default=",".join([
    "PMENV_GAE=tile+PMENV_GAE_U=8", "PMENV_GAE=tile+PMENV_GAE_U=16",
    "PMENV_GAE=tile+PMENV_GAE_U=8+PMENV_GAE_E=1", "PMENV_GAE=tile+PMENV_GAE_U=16+PMENV_GAE_E=1",
    "PMENV_GAE=tile+PMENV_GAE_U=8+PMENV_GAE_E=2", "PMENV_GAE=tile+PMENV_GAE_U=4+PMENV_GAE_E=2",
    "PMENV_GAE=tile+PMENV_GAE_U=4+PMENV_GAE_E=4"]))
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--calls", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda:0")
lib = _abi.load()
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
KN = ("PMENV_GAE", "PMENV_GAE_U", "PMENV_GAE_E", "PMENV_GAE_NW")


def knobs(v):
    d = {}
    for kv in v.split("#")[0].split("+"):
        if "=" in kv:
            k, val = kv.split("=")
            d[k] = val
    return d


out = {}
for shape in a.shapes.split(","):
    T, B = map(int, shape.split("x"))
    g = torch.Generator(device=dev).manual_seed(T + B)
    r = torch.randn(T, B, device=dev, generator=g)
    v = torch.randn(T + 1, B, device=dev, generator=g)
    d = (torch.rand(T, B, device=dev, generator=g) < 0.01).to(torch.uint8)
    bufs = {vn: (torch.empty_like(r), torch.empty_like(r)) for vn in a.variants.split(",")}

    def call(vn):
        for k in KN:
            os.environ.pop(k, None)
        os.environ.update(knobs(vn))
        adv, ret = bufs[vn]
        assert lib.pmenv_gae(P(r), P(v), P(d), P(adv), P(ret), T, B, 0.99, 0.95, st) == 0

    times = {vn: [] for vn in bufs}
    for rd in range(a.rounds):
        for vn in bufs:
            call(vn)
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(a.calls):
                call(vn)
            t1.record()
            torch.cuda.synchronize()
            if rd:
                times[vn].append(t0.elapsed_time(t1) * 1e3 / a.calls)
    first = next(iter(bufs))
    by_u = {}
    for vn, (adv, ret) in bufs.items():
        kv = knobs(vn)                             # same segment (NW x U): same arithmetic
        u = int(kv.get("PMENV_GAE_U", "8")) * int(kv.get("PMENV_GAE_NW", "8"))
        if u in by_u:
            assert torch.equal(adv, by_u[u][0]) and torch.equal(ret, by_u[u][1]), (vn, "not bitwise equal at U", u)
        else:
            by_u[u] = (adv, ret)
        torch.testing.assert_close(adv, bufs[first][0], rtol=1e-5, atol=1e-5)
    alg = T * B * 17 + B * 4
    out[shape] = {vn: {"median_us": round(statistics.median(t), 2), "min_us": round(min(t), 2),
                       "GBs": round(alg / statistics.median(t) / 1e3, 1)} for vn, t in times.items()}
    del r, v, d, bufs
print(json.dumps(out, indent=1))
