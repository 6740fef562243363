"""A/B the replay gather variants (env knobs read at each call) in ONE process,
interleaved rounds; every variant's s / s' must equal the first's bit for bit."""
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
from pmenv import MarketSeries, synth, _abi  # noqa: E402
from pmenv.replay import DeviceReplay  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="base,PMENV_REPLAY_NT=0,PMENV_REPLAY_TPB=512")
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--calls", type=int, default=20)
ap.add_argument("--samples", type=int, default=8192)
a = ap.parse_args()
dev = torch.device("cuda:0")
lib = _abi.load()
B, N, W, H, S = 4096, 30, 50, 256, a.samples
ser = synth.series(2048, 1, N, device=dev)[:, 0].contiguous()
ms = MarketSeries(ser)
rb = DeviceReplay(B, N, W, H, ms)
for h in range(H):
    rb.add(torch.full((B,), W + h, dtype=torch.int32, device=dev), torch.rand(B, N, device=dev), torch.randn(B, device=dev))
h0, e = rb.indices(S, generator=torch.Generator().manual_seed(2))
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = lambda t: ctypes.c_void_p(t.data_ptr())
bufs = {}
for v in a.variants.split(","):
    bufs[v] = [torch.empty(S, N, W, 5, device=dev), torch.empty(S, N, W, 5, device=dev),
               torch.empty(S, N, device=dev), torch.empty(S, device=dev)]
KN = ("PMENV_REPLAY_NT", "PMENV_REPLAY_TPB", "PMENV_REPLAY_LDS", "PMENV_REPLAY_PERSIST", "PMENV_REPLAY_GRID")


def call(v):
    for k in KN:
        os.environ.pop(k, None)
    for kv in v.split("#")[0].split("+"):  # "#k" suffix: the same knobs on another buffer set
        if "=" in kv:
            os.environ[kv.split("=")[0]] = kv.split("=")[1]
    s_, s2, ao, ro = bufs[v]
    rc = lib.pmenv_replay_gather(P(ms.bars), ms.bars.shape[0], N, 5, W, P(rb.days), P(rb.actions), P(rb.rewards), H, B,
                                 P(h0), P(e), S, P(s_), P(s2), P(ao), P(ro), st)
    assert rc == 0


times = {v: [] for v in bufs}
for r in range(a.rounds):
    for v in bufs:
        call(v)
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(a.calls):
            call(v)
        t1.record()
        torch.cuda.synchronize()
        if r:
            times[v].append(t0.elapsed_time(t1) * 1e3 / a.calls)
ref = None
for v, b in bufs.items():
    if ref is None:
        ref = b
    else:
        assert all(torch.equal(x, y) for x, y in zip(b, ref)), v
alg = S * (2 * N * W * 5 * 4 + N * 4 + 4)
print(json.dumps({v: {"median_us": statistics.median(t), "min_us": min(t),
                      "GBs": alg / statistics.median(t) / 1e3} for v, t in times.items()}, indent=1))
