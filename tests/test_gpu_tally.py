"""k_finalize (tally, thresholds, round limits, transitions) on the GPU against the reference's
deterministic KATs (tests/threshold_tests.rs, rfc_compliance_tests.rs:361-372, session.rs:427-524),
using real signed votes so the whole validate-many path runs."""
import numpy as np
import pytest

import coracle
import pyoracle as po
from hashgraph_like_consensus.batch import ProposalConfig, pack_proposals
from scenarios import T0, chain, new_proposal

pytestmark = pytest.mark.gpu
T23 = 2.0 / 3.0

# (n, yes, no, threshold, liveness, gossipsub, max_rounds)
CASES = [
    (3, 2, 1, T23, False, True, 2), (3, 1, 2, T23, True, True, 2), (2, 1, 1, T23, True, True, 2),
    (2, 2, 0, T23, False, True, 2), (5, 3, 2, 0.9, True, True, 2), (5, 2, 1, 0.5, True, True, 2),
    (4, 2, 0, T23, True, True, 2), (4, 2, 2, T23, False, True, 2), (4, 2, 2, T23, True, True, 2),
    (1, 0, 1, T23, True, True, 2), (1, 1, 0, T23, False, True, 2), (6, 2, 2, T23, True, True, 2),
    (9, 6, 0, T23, True, False, 0), (9, 5, 2, T23, True, False, 0), (9, 4, 3, T23, False, False, 0),
    (10, 7, 0, T23, True, False, 0), (10, 3, 4, T23, True, False, 0), (5, 2, 2, 0.75, False, False, 3),
    (5, 2, 2, 0.75, False, False, 5), (100, 40, 27, T23, True, True, 2), (7, 3, 3, T23, True, False, 0),
]


def test_gpu_tally_kats(engine):
    props, cfgs, expect = [], [], []
    for c, (n, yes, no, t, live, goss, mr) in enumerate(CASES):
        p = new_proposal(1000 + c, n, liveness=live)
        chain(p, [(k, k < yes) for k in range(yes + no)], vid0=100 * c + 1)
        cfg = po.ConsensusConfig(t, mr, goss, live)
        props.append(p)
        cfgs.append(ProposalConfig(t, mr, goss))
        expect.append(po.from_proposal(p, cfg, T0 + 5))
    batch, desc = pack_proposals(props, cfgs)
    res, vst, _, _ = engine.validate_proposals(batch, desc, T0 + 5)
    cres, cvst, _, _ = coracle.validate_proposals(batch, desc, T0 + 5, threads=4)
    assert np.array_equal(res, cres) and np.array_equal(vst, cvst)
    for k, e in enumerate(expect):
        assert int(res[k]["status"]) == e.status, CASES[k]
        assert int(res[k]["transition"]) == e.transition, CASES[k]
        if e.status == po.OK:
            assert int(res[k]["yes"]) == e.yes and int(res[k]["total"]) == e.total
    # the set must exercise every transition and the round-limit rejection
    assert {int(r["transition"]) for r in res} == {0, 1, 2}
    assert po.MAX_ROUNDS_EXCEEDED in {int(r["status"]) for r in res}
