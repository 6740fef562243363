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
    # which kernel time the headline frac divides by: the event mean, or the unbracketed step
    # time when the event mean exceeds it (then frac == frac_step); the event figure stays
    assert r["frac_source"] and abs(r["frac_event"] - r["achieved_event"] / r["peak"]) < 1e-9
    if r["kernel_avg_us"] > d["ms_per_step"] * 1e3:
        assert r["frac_source"].startswith("ms_per_step") and r["frac"] == r["frac_step"]
    else:
        assert r["frac_source"].startswith("kernel_avg_us") and r["frac"] == r["frac_event"]
    assert d["library"]["sha256"] and d["library"]["path"].endswith("libpmenv.so")
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


def _two_ranks(*extra):
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--dist-backend", "gloo", "--steps", "8", "--warmup", "2", "--alt-steps", "0", *extra]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip().startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_two_ranks_rehearsal():
    """The driver's N > 1 launch (torch.distributed.run, one process per rank) with both
    ranks on the one GPU over gloo (RCCL refuses two ranks on a device), by default: the
    north star's strong-scaled workload, 65,536 envs in total sharded 32,768 per rank,
    value = all envs' steps over the max-over-ranks time, the moments all-reduce
    recorded, parity on every rank, the weak-scaled workload beside it under alt_weak."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = _two_ranks("--alt-weak-steps", "4")
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["global_envs"] == 65536 and d["config"]["envs_per_gpu"] == 32768
    assert d["config"]["per_rank"]["envs"] == 32768 and "step_path" in d["config"]["per_rank"]
    assert abs(d["value"] - 65536 * 1e3 / d["ms_per_step"]) <= 1e-6 * d["value"]
    assert d["collective"]["backend"] == "gloo" and d["collective"]["count_all_ranks"] > 0
    assert d["parity_sample"]["obs_bit_exact_all_ranks"] is True
    assert d["parity_sample"]["reward_max_rel_all_ranks"] <= 1e-6
    assert d["cpu_baseline"] is None                     # rank 0 at N = 1 only
    w = d["alt_weak"]
    assert w["scaling"] == "weak" and w["envs_per_gpu"] == 65536 and w["global_envs"] == 131072
    assert w["value"] > 0 and w["nonfinite_envs"] == 0


def test_bench_two_ranks_weak():
    """--envs-per-gpu keeps the weak-scaled form: per-rank work fixed as N grows."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = _two_ranks("--envs-per-gpu", "2048")
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["config"]["global_envs"] == 4096
    assert abs(d["value"] - 2 * 2048 * 1e3 / d["ms_per_step"]) <= 1e-6 * d["value"]
    assert d["parity_sample"]["obs_bit_exact_all_ranks"] is True
