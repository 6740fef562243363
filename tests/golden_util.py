"""Loading and replaying the golden vectors of tests/golden (made by gen_golden.py
from the reference env itself)."""
import glob
import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def cases():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz"))
                  if not p.endswith(("reward_module.npz", "trainer_reward.npz", "onpolicy_driver.npz")))


def load(name):
    d = np.load(os.path.join(GOLDEN_DIR, name + ".npz"))
    g = {k: d[k] for k in d.files}
    g["meta"] = json.loads(str(g["meta"]))
    return g


def close_channel(g):
    """The series' close channel (the F = 5 cases predate the meta field: OHLC's 3)."""
    return g["meta"].get("close_channel", 3)


def load_driver():
    """tests/golden/onpolicy_driver.npz: train/on_policy.py's env call sequence on the
    reference (gen_golden.driver_vectors)."""
    d = np.load(os.path.join(GOLDEN_DIR, "onpolicy_driver.npz"))
    g = {k: d[k] for k in d.files}
    for k in list(g):
        if k == "meta" or k.endswith("info_types"):
            g[k] = json.loads(str(g[k]))
    return g


def window(g, i):
    """window_i = series[:, i:i+W] as the [1, N, W, F] float32 obs batch."""
    W = g["meta"]["W"]
    return np.ascontiguousarray(g["series"][None, :, i:i + W, :])


def bar(g, i):
    """The market channels of the day appended at loop index i: series[:, i+W-1, :F-1]."""
    W, F = g["meta"]["W"], g["meta"]["F"]
    return np.ascontiguousarray(g["series"][None, :, i + W - 1, :F - 1])


def tolerances(g):
    """(rtol on value/ret, abs floor on reward) — SURVEY.md §8c parity criteria.
    fp64 goldens: 1e-6 relative (north star). fp32 goldens differ from an f64
    computation by fp32 rounding of the reference itself."""
    if g["meta"]["dtype"] == "f64":
        return 1e-6, 1e-9
    return 2e-5, 2e-6


def finite_prefix(g):
    """Steps before the fp32 reference overflowed (rawpos actions compound x~15/day)."""
    v = g["values"]
    bad = np.nonzero(~np.isfinite(v))[0]
    return len(v) if bad.size == 0 else int(bad[0])
