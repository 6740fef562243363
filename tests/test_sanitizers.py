"""Host sanitizers: the CPU restatement and the host emulation of the
HIP path's two in-place window-advance schedules (the flat stream with its halo; one
workgroup per env), built with AddressSanitizer + UndefinedBehaviorSanitizer
(oracle/sanitize/build.sh) and run on random inputs in every mode. The emulation runs
the workgroups in a random order with every store visible at once and checks that no
workgroup reads a chunk another one has already stored (read-before-write) and that
the in-place result equals an out-of-place advance. CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_asan_ubsan_oracle_and_schedule_emulation(tmp_path):
    exe = str(tmp_path / "sanitize_bin")
    b = subprocess.run(["sh", os.path.join(ROOT, "oracle", "sanitize", "build.sh"), exe],
                       capture_output=True, text=True)
    if b.returncode != 0 and "asan" in (b.stderr + b.stdout).lower():
        pytest.skip(f"sanitizer runtime unavailable: {b.stderr[-300:]}")
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", OMP_NUM_THREADS="4")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "sanitize ok" in r.stdout
