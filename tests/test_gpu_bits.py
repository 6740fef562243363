"""Bit fingerprints of the env step against the round-4 library of record
(tools/step_bits.py -> tests/golden/step_bits.json, written by the r04l build): windows,
rewards and values after six steps with raw (softmax) and simplex actions, at every
scalar-step form (N = 8 / 16 packed, 30 / 64 register, 100 / 300 / 500 packed strided),
every reward kind (commission on one) and every step path the shape takes. A regression
anchor for rewrites that must not move a bit; the numerics themselves are pinned against
the oracle and the reference's goldens elsewhere. Needs an MI355X."""
import json
import os
import sys

import pytest
import torch

import golden_util as gu

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(DEV)


def test_gpu_step_bits_match_the_library_of_record():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import step_bits
    want = json.load(open(os.path.join(gu.GOLDEN_DIR, "step_bits.json")))
    got = step_bits.fingerprints(str(DEV))
    assert set(got) == set(want)
    bad = sorted(k for k in want if got[k] != want[k])
    assert not bad, f"{len(bad)} of {len(want)} fingerprints moved, e.g. {bad[:5]}"
