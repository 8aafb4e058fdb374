"""Golden fixtures (tests/golden/, made by make_golden.py with both oracles agreeing) are
reproduced bit-exactly by the C restatement; the GPU side is in test_gpu_scenarios.py."""
import os

import numpy as np
import pytest

import coracle
from golden_io import fixtures, load

FIX = fixtures()


def test_fixtures_present():
    names = {os.path.basename(f) for f in FIX}
    assert "config1_gossipsub_3_voters.npz" in names and "config5_byzantine_small.npz" in names


@pytest.mark.parametrize("path", FIX, ids=[os.path.basename(f) for f in FIX])
def test_c_oracle_reproduces_golden(path):
    batch, desc, now, exp = load(path)
    res, vst, vrs, rec = coracle.validate_proposals(batch, desc, now, threads=2)
    assert np.array_equal(res, exp["results"])
    assert np.array_equal(vst, exp["vote_status"])
    assert np.array_equal(vrs, exp["vote_reason"])
    assert np.array_equal(rec, exp["recovered"])


def test_config1_reaches_consensus():
    batch, desc, now, exp = load([f for f in FIX if "config1" in f][0])
    r = exp["results"][0]
    assert int(r["status"]) == 0 and int(r["total"]) == 3
