"""SURVEY.md §8d config 5 built by product code on the device (hlc_synth_byzantine_device):
1/3 Byzantine votes over 17 mutation kinds, each built to have one outcome.

* The kinds the device applies equal the plan recomputed on the host from the seed.
* The GPU's per-vote statuses / scheme reasons and per-proposal first errors equal the outcomes
  the plan is built to have (byzantine.expectations, no oracle) -- what bench.py asserts before it
  times the mix -- AND equal the C oracle's on the same mutated bytes, bit for bit.
"""
import numpy as np
import pytest

import coracle
from hashgraph_like_consensus import byzantine, synth
from hashgraph_like_consensus.device import DeviceBatch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("P,start", [(1200, 0), (300, 777)])
def test_gpu_config5_device_mutator(engine, P, start):
    V = 64
    seed = synth.config_seed(5)
    db = DeviceBatch.synthetic(engine, P, V, V, True, seed, start_proposal=start)
    kinds = db.make_byzantine(engine, seed, start)
    assert np.array_equal(kinds, byzantine.plan(seed, start, P, V))
    frac = float((kinds != 0).mean())
    assert 0.30 < frac < 0.37, frac
    assert set(np.unique(kinds).tolist()) == set(range(18))
    engine.validate_proposals_device(db)
    db.torch.cuda.synchronize()
    res, st = db.results_numpy(), db.status_numpy()
    rs = db.reason[: db.n].cpu().numpy()
    vst, vrs, pst, bad, yes, total = byzantine.expectations(kinds, V, db.choice_numpy())
    assert np.array_equal(st, vst), np.nonzero(st != vst)[0][:10]
    sch = st == byzantine.SCHEME
    assert np.array_equal(rs[sch], vrs[sch])
    assert np.array_equal(res["status"], pst), np.nonzero(res["status"] != pst)[0][:10]
    assert np.array_equal(res["bad_index"], bad)
    ok = pst == 0
    assert np.array_equal(res["yes"][ok], yes[ok]) and np.array_equal(res["total"][ok], total[ok])
    # every proposal-level class the plan can produce is present
    assert {0, 2, 3, 4, 5, 6, 7, 8, 9, 11, 12, 13} <= set(np.unique(pst).tolist())
    # bit for bit against the C oracle on the same mutated bytes
    hb, hd, _ = db.to_host()
    cres, cvst, cvrs, _ = coracle.validate_proposals(hb, hd, db.now, threads=16)
    assert np.array_equal(st, cvst) and np.array_equal(rs, cvrs)
    assert np.array_equal(res, cres)
