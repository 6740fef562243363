"""Bit fingerprints of the batched reward (f2, agent/pg/pg.py:40-82) — the reward, the
per-row returns and the gradient — over deterministic numpy inputs at every row form
(the quad form for N <= 64, EPL 8 / 16; the wave form above), reward kind and norm mode,
with simplex rows, negative rows and a NaN row among them. Written by the library of
record into tests/golden/f2_bits.json; tests/test_gpu_trainer.py checks that later
libraries reproduce them bit for bit (a regression anchor for kernel rewrites that must
not change a single bit; the numerics themselves are pinned against the oracle and the
reference's autograd elsewhere).

    python tools/f2_bits.py > tests/golden/f2_bits.json
    python tools/f2_bits.py --lib tools/libpmenv_old.so > old.json     # another build
    python tools/f2_bits.py --check old.json                            # exit 1 if a bit moved
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))

SHAPES = [(65536, 30), (16384, 30), (4096, 30), (1000, 7), (333, 17), (4096, 64), (8192, 500), (8, 200)]
KINDS = ["log_returns", "returns", "sharpe_ratio"]
NORMS = ["global_or", "row_or", "none"]


def inputs(B, N, case):
    rng = np.random.default_rng(B * 131 + N * 7 + case)
    a = rng.standard_normal((B, N)).astype(np.float32)
    if case == 1:                                   # simplex rows (and a batch sum far from 1)
        a = np.abs(a) / np.abs(a).sum(1, keepdims=True)
    if case == 2:                                   # mixed: simplex rows, negative rows, a NaN row
        a[::2] = np.abs(a[::2]) / np.abs(a[::2]).sum(1, keepdims=True)
        a[B // 3] = np.nan
    v = (25000.0 * np.exp(0.1 * rng.standard_normal(B))).astype(np.float32)
    p = (1.0 + 0.01 * rng.standard_normal((B, N))).astype(np.float32)
    return a.astype(np.float32), v, p


def fingerprints(dev="cuda:0"):
    import torch
    from pmenv.trainer import batch_reward
    out = {}
    for B, N in SHAPES:
        for case in range(3):
            a_np, v_np, p_np = inputs(B, N, case)
            for kind in KINDS:
                for norm in NORMS:
                    a = torch.tensor(a_np, device=dev).reshape(B, N, 1).requires_grad_(True)
                    r, ret = batch_reward(a, torch.tensor(v_np, device=dev),
                                          torch.tensor(p_np, device=dev).reshape(B, N, 1),
                                          reward=kind, norm=norm, return_ret=True)
                    (2.0 * r).backward()
                    h = hashlib.sha256()
                    for t in (r.detach().reshape(1), ret.detach(), a.grad):
                        h.update(t.contiguous().cpu().numpy().tobytes())
                    out[f"{B}x{N}/{case}/{kind}/{norm}"] = h.hexdigest()[:32]
    return out


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", help="load this libpmenv build instead of the in-tree one")
    ap.add_argument("--check", help="compare against these fingerprints instead of printing")
    a = ap.parse_args()
    if a.lib:
        from pmenv import _abi
        _abi.LIB_PATH = os.path.abspath(a.lib)
    got = fingerprints()
    if not a.check:
        print(json.dumps(got, indent=1, sort_keys=True))
        sys.exit(0)
    want = json.load(open(a.check))
    bad = sorted(k for k in want if got.get(k) != want[k])
    print(f"f2_bits: {len(want) - len(bad)} of {len(want)} fingerprints equal" + (f"; moved: {bad[:8]}" if bad else ""))
    sys.exit(1 if bad or set(got) != set(want) else 0)
