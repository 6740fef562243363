"""Where the cache-resident relay step (step_relay_kernel, BASELINE config 2 and config 4's
8-GPU share) spends its time: the tools build's own instantiation of the product kernel
(PMENV_RELAY_STAMPS: step_relay_kernel<..., ANY = 2>, the product's code plus
relay_clock, step_relay.h) reads s_memrealtime (100 MHz, 10 ns ticks) in thread 0 of every
workgroup at each phase of its role — once the phase's last load has returned, or ([5], [2]
of a scalar block) once the wave's stores have completed — and stores the stamps at the
workgroup's end:

  tile   [0] entry  [1] window chunks, bar, counter and first w' read returned  [2] wave 0's
         w' all arrived (after polls)  [3] every wave staged (barrier)  [4] stores issued
         [5] stores completed
  scalar [0] entry  [1] relay words published (list read)  [2] state written

For each of kStampSlots consecutive steps (in place, back to back after a warm-up) the
stamps are taken relative to the step's first workgroup entry; the summary is the median
over the steps of each statistic. The product library runs beside it (HIP events over K
steps) and so does the tools instantiation with its stamps not stored, to size the perturbation.

    python tools/relay_stamps.py [--shapes 8192x30,4096x30]   # prints one JSON object
"""
import argparse
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

K = 200
TICK_NS = 10.0
RELAY = 4                     # PMENV_STEP_PATH_RELAY


def pct(x, q):
    return float(np.percentile(x, q)) if len(x) else float("nan")


def analyse(st, n_slots):
    """st: [slots][max_wg][8] int64 ticks. Returns per-step statistics (ns)."""
    steps = []
    for s in range(n_slots):
        a = st[s]
        used = a[:, 0] != 0
        a = a[used]
        if len(a) == 0:
            continue
        tile = a[:, 5] != 0
        scal = ~tile & (a[:, 1] != 0)
        t0 = a[:, 0].min()
        A = (a - t0) * TICK_NS
        T, S = A[tile], A[scal]
        d = {
            "workgroups": int(len(a)), "tiles": int(tile.sum()), "scalar_blocks": int(scal.sum()),
            "span_ns": float(A[:, 5].max() if tile.any() else 0.0),
            "scalar_entry_max_ns": float(S[:, 0].max()) if len(S) else None,
            "scalar_words_published_p50_ns": pct(S[:, 1], 50) if len(S) else None,
            "scalar_words_published_max_ns": float(S[:, 1].max()) if len(S) else None,
            "scalar_state_written_max_ns": float(S[:, 2].max()) if len(S) else None,
            "tile_entry_p10_ns": pct(T[:, 0], 10), "tile_entry_p50_ns": pct(T[:, 0], 50),
            "tile_entry_p90_ns": pct(T[:, 0], 90), "tile_entry_max_ns": float(T[:, 0].max()),
            "tile_exit_p50_ns": pct(T[:, 5], 50), "tile_exit_max_ns": float(T[:, 5].max()),
            "tile_life_mean_ns": float((T[:, 5] - T[:, 0]).mean()),
            "tile_load_mean_ns": float((T[:, 1] - T[:, 0]).mean()),
            "tile_wait_mean_ns": float((T[:, 2] - T[:, 1]).mean()),
            "tile_wait_p99_ns": pct(T[:, 2] - T[:, 1], 99),
            "tiles_waiting_frac": float(((T[:, 2] - T[:, 1]) > 2 * TICK_NS).mean()),
            "tile_barrier_mean_ns": float((T[:, 3] - T[:, 2]).mean()),
            "tile_compose_issue_mean_ns": float((T[:, 4] - T[:, 3]).mean()),
            "tile_store_drain_mean_ns": float((T[:, 5] - T[:, 4]).mean()),
            # waves-0 in flight: the tiles' summed lifetimes over the span (per CU: / 256)
            "tiles_in_flight_mean": float((T[:, 5] - T[:, 0]).sum() / max(A[:, 5].max(), 1.0)),
            # the stream's ramp and drain: the span before the first 10 % of tiles entered, and
            # after the last tile entered
            "ramp_ns": pct(T[:, 0], 10), "tail_after_last_entry_ns": float(A[:, 5].max() - T[:, 0].max()),
        }
        steps.append(d)
    out = {}
    for k in steps[0]:
        vals = [x[k] for x in steps if x[k] is not None]
        out[k] = statistics.median(vals) if vals else None
    out["steps"] = len(steps)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="8192x30,4096x30")
    args = ap.parse_args()
    torch.cuda.set_device(ab.DEV)
    prod = ab.load(os.path.join(ROOT, "pm-rl_amd", "pmenv", "libpmenv.so"))
    tools = ab.load(os.path.join(ROOT, "tools", "libpmenv_ab.so"))
    tools.pmenv_tools_relay_stamps.restype = ctypes.c_int
    tools.pmenv_tools_relay_stamps.argtypes = [ctypes.c_void_p]
    sl, mw = ctypes.c_uint32(), ctypes.c_uint32()
    tools.pmenv_tools_relay_stamp_dims(ctypes.byref(sl), ctypes.byref(mw))
    n_slots, max_wg = sl.value, mw.value
    out = {"K": K, "tick_ns": TICK_NS}
    for shape in args.shapes.split(","):
        B, N = (int(x) for x in shape.split("x"))
        os.environ["PMENV_RELAY_STAMPS"] = "1"
        et = ab.Env(tools, B, N, 50, RELAY, False)
        os.environ.pop("PMENV_RELAY_STAMPS", None)
        ep = ab.Env(prod, B, N, 50, RELAY, False)
        paths = {"product": prod.pmenv_step_path(ep.h).decode(), "tools": tools.pmenv_step_path(et.h).decode()}
        for e in (ep, et):
            for _ in range(50):
                e.step()
        ev = {"product": [], "tools_clocks_unstored": []}
        for _ in range(5):
            ev["product"].append(ab.timed(ep.step, K))
            ev["tools_clocks_unstored"].append(ab.timed(et.step, K))
        buf = torch.zeros(n_slots * max_wg * 8, dtype=torch.int64, device=ab.DEV)
        torch.cuda.synchronize()
        assert tools.pmenv_tools_relay_stamps(ctypes.c_void_p(buf.data_ptr())) == 0
        stamped = ab.timed(et.step, n_slots)           # one launch per slot, back to back
        assert tools.pmenv_tools_relay_stamps(None) == 0
        torch.cuda.synchronize()
        st = buf.view(n_slots, max_wg, 8).cpu().numpy()
        res = {"paths": paths, "event_us_per_step": {k: statistics.median(v) for k, v in ev.items()},
               "stamped_event_us_per_step": stamped}
        res.update(analyse(st, n_slots))
        out[shape] = res
        print(shape, json.dumps(res), file=sys.stderr, flush=True)
        ep.close()
        et.close()
        del buf
    print(json.dumps(out))


if __name__ == "__main__":
    main()
