"""Host sanitizers: the CPU restatement and the host emulation of the
HIP path's in-place schedules, built with AddressSanitizer + UndefinedBehaviorSanitizer
(oracle/sanitize/build.sh) and run on random inputs in every mode:
  * the flat stream with its halo, one workgroup per env, and the flat one-launch step —
    workgroups in a random order with every store visible at once; no workgroup reads a
    chunk another one has already stored, and the in-place result equals an out-of-place
    advance;
  * the relayed step (step_relay.h) — scalar blocks and tiles interleaved at random, a tile
    runnable only once its rows' relay words carry the step's epoch or, past its polls, giving
    up and running its rows' scalar-step units under their claims, through the epoch's wrap,
    caller edits, a state write and a step of another path, in blockIdx order, any order, one
    resident workgroup and tiles first — no deadlock, every env stepped once from its pre-step
    state, the product's bits; every staged row fits the tile's threads and every LDS / halo /
    counter index its buffer; without the fallback, one resident in a non-monotone order must
    deadlock (the detection's negative control);
  * the one-pass look-back GAE — workgroups publishing and composing in a random order under
    the flag waits, on an exact-size workspace holding garbage or the previous call's flags;
  * an address audit of the halo copy for every scalar-step grid and of the tools build's
    advance_flat_direct_kernel at the shapes of profiles/ab_r03/direct_r03d.err.
CPU only."""
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
