"""The C ABI driven from plain C (tests/c_abi/c_abi_step.c: no Python, no torch — the
shape of a non-Python caller): device-side synthetic workload, every advance-step
implementation in place through the ring wrap, each step checked against the CPU
restatement. Needs an MI355X."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "c_abi", "c_abi_step")


@pytest.mark.parametrize("shape", [(600, 30, 50, 60), (301, 4, 30, 40), (3, 64, 47, 52)],
                         ids=lambda s: "x".join(map(str, s)))
def test_gpu_c_caller_every_step_path(shape):
    if not os.path.exists(BIN):
        pytest.fail("tests/c_abi/c_abi_step is not built (pm-rl_amd/build.py build_c_abi_test)")
    out = subprocess.run([BIN, *map(str, shape)], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("c_abi ok")]
    assert [l.split()[2] for l in lines] == ["auto", "flat", "one_launch", "two_launch"], out.stdout
    flat = next(l for l in lines if l.split()[2] == "flat")
    assert flat.count("step_flat_kernel") == 2
