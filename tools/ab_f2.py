"""A/B of the batched reward (f2: PG._reward / A2C._loss, agent/pg/pg.py:40-82) forward and
backward between the product library and the tools build with PMENV_BR_* knobs (read at
call time by the tools build only), in ONE process, interleaved rounds; the outputs are
compared bit for bit (reward, per-row returns, gradient).

    python tools/ab_f2.py --knobs PMENV_BR_RELAY=1 --shapes 65536x30,16384x30,4096x30
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402
from pmenv import _abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--knobs", default="PMENV_BR_RELAY=1")
ap.add_argument("--shapes", default="65536x30,16384x30,4096x30")
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--calls", type=int, default=100)
ap.add_argument("--kind", default="log_returns")
a = ap.parse_args()
for kv in a.knobs.split(","):
    if kv:
        k, v = kv.split("=", 1)
        os.environ[k] = v
dev = torch.device("cuda:0")
libs = {}
for name, path in (("product", os.path.join(ROOT, "pm-rl_amd/pmenv/libpmenv.so")),
                   ("tools", os.path.join(ROOT, "tools/libpmenv_ab.so"))):
    lib = ctypes.CDLL(path)
    for n, res, args in _abi.SIGNATURES:
        fn = getattr(lib, n, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    libs[name] = lib
kind = _abi.REWARD_KINDS[a.kind]
out = {}
for shp in a.shapes.split(","):
    B, N = (int(x) for x in shp.split("x"))
    g = torch.Generator(device=dev).manual_seed(B + N)
    act = torch.randn(B, N, device=dev, generator=g)
    v = 25000 * torch.exp(0.1 * torch.randn(B, device=dev, generator=g))
    p = 1 + 0.01 * torch.randn(B, N, device=dev, generator=g)
    go = torch.ones((), device=dev)
    res = {}
    for name, lib in libs.items():
        work = torch.empty(lib.pmenv_batch_reward_workspace(B) // 8, dtype=torch.float64, device=dev)
        rew = torch.empty((), device=dev)
        grad = torch.empty(B, N, device=dev)
        res[name] = (lib, work, rew, grad)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def fwd(x):
        lib, work, rew, _ = x
        rc = lib.pmenv_batch_reward_forward(act.data_ptr(), v.data_ptr(), p.data_ptr(), B, N, kind, 0, 1.0,
                                            work.data_ptr(), rew.data_ptr(), None, st)
        assert rc == 0

    def bwd(x):
        lib, work, _, grad = x
        rc = lib.pmenv_batch_reward_backward(act.data_ptr(), v.data_ptr(), p.data_ptr(), B, N, kind, 1.0,
                                             work.data_ptr(), go.data_ptr(), grad.data_ptr(), st)
        assert rc == 0
    for x in res.values():
        fwd(x)
        bwd(x)
    torch.cuda.synchronize()
    bits = {n: bool(torch.equal(x[2], res["product"][2]) and torch.equal(x[3], res["product"][3]))
            for n, x in res.items()}
    times = {n: {"fwd": [], "fwd_bwd": []} for n in res}
    for r in range(a.rounds):
        for n in (list(res) if r % 2 == 0 else list(reversed(list(res)))):
            x = res[n]
            for mode in ("fwd", "fwd_bwd"):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.calls):
                    fwd(x)
                    if mode == "fwd_bwd":
                        bwd(x)
                e1.record()
                torch.cuda.synchronize()
                times[n][mode].append(e0.elapsed_time(e1) * 1e3 / a.calls)
    line = {n: {m: statistics.median(t) for m, t in d.items()} for n, d in times.items()}
    out[shp] = {"us_per_call": line, "bits_equal": bits}
    for n in res:
        print(f"# f2 {shp} {a.kind} {n:8s} fwd {line[n]['fwd']:7.2f} us  fwd+bwd {line[n]['fwd_bwd']:7.2f} us "
              f"bits_equal={bits[n]}", file=sys.stderr, flush=True)
print(json.dumps(out, indent=1))
