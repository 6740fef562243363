"""Where config 1's step (1 x 5 x 50 x 5, step_small_kernel<256, 8, true>) spends its time:
the tools build's small_stamp_kernel (PMENV_SMALL_ABL) stamps s_memrealtime at each phase
of the step, with timing-only ablations, and the product library's kernel runs beside it.
Run under `rocprofv3 --kernel-trace --stats` for the kernels' durations (the stamps cover
only the time the first wave runs).

Phases (thread 0, 10 ns ticks): [0] entry, [1] scalar step up to w' done (its loads
returned), [2] own window loads returned, [3] after the barrier, [4] window stores issued,
[5] tail done, [6] own stores acknowledged; [7] the last wave's entry.

    python tools/small_stamps.py          # prints one JSON object
"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ab_r05 as ab  # noqa: E402

K = 1000
LEGS = [("product", None), ("stamped", 0), ("no_scalar", 2), ("no_window", 4), ("neither", 6), ("no_tail", 16),
        ("empty", 8)]
NAMES = ["scalar_done", "loads_done", "barrier", "stores_issued", "tail_done", "stores_acked"]


def main():
    torch.cuda.set_device(ab.DEV)
    prod = ab.load(ab.LIBS["r05"])
    tools = ab.load(os.path.join(ROOT, "tools", "libpmenv_ab.so"))
    tools.pmenv_tools_small_stamps.restype = ctypes.c_int
    tools.pmenv_tools_small_stamps.argtypes = [ctypes.c_void_p]
    out = {"K": K}
    for name, abl in LEGS:
        if abl is None:
            os.environ.pop("PMENV_SMALL_ABL", None)
            lib = prod
        else:
            os.environ["PMENV_SMALL_ABL"] = str(abl)
            lib = tools
        e = ab.Env(lib, 1, 5, 50, 0, False)        # AUTO: the register step
        path = lib.pmenv_step_path(e.h).decode()
        for _ in range(50):
            e.step()
        us = ab.timed(e.step, K)
        res = {"path": path, "event_us_per_step": us}
        if abl is not None:
            st = np.zeros(1024 * 8, np.uint64)
            assert tools.pmenv_tools_small_stamps(st.ctypes.data) == 0
            st = st.reshape(1024, 8).astype(np.int64)
            if abl != 8:
                d = (st[:, :7] - st[:, :1]) * 10        # ns from entry
                for i, n in enumerate(NAMES):
                    res[n + "_ns"] = float(np.median(d[:, i + 1]))
            res["last_wave_entry_ns"] = float(np.median((st[:, 7] - st[:, 0]) * 10))
        e.close()
        out[name] = res
        print(name, json.dumps(res), file=sys.stderr, flush=True)
    os.environ.pop("PMENV_SMALL_ABL", None)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
