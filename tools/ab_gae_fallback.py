"""The look-back GAE's forward-progress fallback on hardware: the product's pmenv_gae_ex
against the tools build's SPIN = 0 form of the same kernel (PMENV_GAE=lbfb: a wave takes
the fallback — computes a later chunk's map itself — on the first poll that finds its flag
missing, so the fallback runs on every early-dispatched chunk), at the shapes the look-back
pass takes. Checks the adv / ret bitwise equal and reports the time of each.

    PMENV_GAE=lbfb python tools/ab_gae_fallback.py
"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402

import ab_r05 as ab  # noqa: E402


def main():
    assert os.environ.get("PMENV_GAE") == "lbfb"
    torch.cuda.set_device(ab.DEV)
    libs = {"product": ab.load(ab.LIBS["r05"]), "fallback": ab.load(os.path.join(ROOT, "tools", "libpmenv_ab.so"))}
    P = ctypes.c_void_p
    out = {}
    for (T, B) in ((4096, 512), (2048, 4096), (16384, 64), (1000, 200), (513, 3), (700, 67)):
        g = torch.Generator(ab.DEV).manual_seed(T + B)
        r = torch.randn(T, B, device=ab.DEV, generator=g)
        v = torch.randn(T + 1, B, device=ab.DEV, generator=g)
        d = (torch.rand(T, B, device=ab.DEV, generator=g) < 0.01).to(torch.uint8)
        res, times = {}, {}
        for n, lib in libs.items():
            ws = lib.pmenv_gae_workspace(T, B)
            work = torch.empty(max(ws // 8, 1), dtype=torch.float64, device=ab.DEV)
            adv, ret = torch.empty(T, B, device=ab.DEV), torch.empty(T, B, device=ab.DEV)

            def call(lib=lib, work=work, ws=ws, adv=adv, ret=ret):
                assert lib.pmenv_gae_ex(P(r.data_ptr()), P(v.data_ptr()), P(d.data_ptr()), P(adv.data_ptr()),
                                        P(ret.data_ptr()), T, B, 0.99, 0.95, P(work.data_ptr()), ws,
                                        ab.stream()) == 0
            for _ in range(5):
                call()
            times[n] = statistics.median(ab.timed(call, 50) for _ in range(5))
            torch.cuda.synchronize()
            res[n] = (adv.clone(), ret.clone())
        key = f"{T}x{B}"
        out[key] = {"product_us": times["product"], "fallback_us": times["fallback"],
                    "bitwise_equal": bool(torch.equal(res["product"][0], res["fallback"][0]) and
                                          torch.equal(res["product"][1], res["fallback"][1]))}
        print(key, json.dumps(out[key]), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
