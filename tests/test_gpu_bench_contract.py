"""bench.py's output contract, on a small workload: one JSON line on stdout with the
driver's keys, the roofline and cpu_baseline objects, a parity record against the CPU
restatement, and no PMENV_* knob. Runs bench.py as a child process (fresh GPU context).
Needs an MI355X."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra, env=None):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--envs-per-gpu", "2048", "--steps", "8", "--warmup", "2",
           "--alt-steps", "4", "--cpu-sample-envs", "256", "--cpu-budget-s", "0.5", "--parity-envs", "256", *extra]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)


def test_bench_prints_the_contract_line():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    p = _run()
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 8 and d["warmup"] == 2 and d["higher_is_better"] is True
    assert d["value"] > 0 and abs(d["value"] - 2048 * 1e3 / d["ms_per_step"]) <= 1e-6 * d["value"]
    assert d["knobs"] == {}
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert 0 < r["achieved"] and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-9
    assert r["l3_resident"] is True                     # a 61 MB window sits in the Infinity Cache
    c = d["cpu_baseline"]
    assert c["value"] > 0 and c["cores"] >= 1 and c["kind"] == "port" and c["sample"]
    assert d["parity_sample"]["obs_bit_exact"] is True
    assert d["reward_mae"] <= 1e-6


def test_bench_refuses_a_knob():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, PMENV_ONE="all")
    p = _run(env=env)
    assert p.returncode != 0 and "PMENV_" in (p.stderr + p.stdout)
