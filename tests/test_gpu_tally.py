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


U32 = 2**32 - 1


def test_gpu_round_limit_u32_edges(engine):
    """k_finalize at the u32 edges of check_round_limit (session.rs:306-344): the P2P ceil(2n/3) cap
    computed in u32 wraps for n >= 2^31 (release build), so 5 votes against n = 2^31 + 5 exceed a
    cap of 4 while 4 votes pass; n = u32::MAX gives a cap of 1431655765; Gossipsub with an explicit
    max_rounds of 1 fails as soon as a vote moves the session to round 2."""
    specs = [  # (n, votes, gossipsub, max_rounds)
        (2**31 + 5, 5, False, 0), (2**31 + 5, 4, False, 0), (2**31 + 6, 4, False, 0), (U32, 6, False, 0),
        (U32, 3, False, U32), (U32, 3, False, 2), (5, 2, True, 1), (5, 2, True, 2),
    ]
    props, cfgs, expect = [], [], []
    for c, (n, k, goss, mr) in enumerate(specs):
        p = new_proposal(3000 + c, n)
        chain(p, [(j, j % 2 == 0) for j in range(k)], vid0=500 * c + 1)
        props.append(p)
        cfgs.append(ProposalConfig(T23, mr, goss))
        expect.append(po.from_proposal(p, po.ConsensusConfig(T23, mr, goss, True), T0 + 5))
    batch, desc = pack_proposals(props, cfgs)
    res, vst, _, _ = engine.validate_proposals(batch, desc, T0 + 5)
    cres, cvst, _, _ = coracle.validate_proposals(batch, desc, T0 + 5, threads=4)
    assert np.array_equal(res, cres) and np.array_equal(vst, cvst)
    got = [int(r["status"]) for r in res]
    assert got == [e.status for e in expect]
    mre = po.MAX_ROUNDS_EXCEEDED
    assert got == [mre, po.OK, po.OK, po.OK, po.OK, mre, mre, po.OK], got


def test_gpu_stream_update_round_saturates(engine):
    """update_round's saturating_add (session.rs:364; the reference's test at session.rs:674-699) in
    the streaming kernel: P2P sessions already at round u32::MAX - 1 / u32::MAX with an explicit
    max_rounds of u32::MAX accept their votes and stay at u32::MAX (no wrap to 0); with the ceil(2n/3)
    cap (max_rounds 0) the saturated projection exceeds it and the session fails."""
    import stream_oracle as so
    from stream_cases import device_inputs, run_oracle, sessions_array

    sessions, votes, vs = [], [], []
    for c, (start, mr) in enumerate([(U32 - 1, U32), (U32, U32), (U32 - 1, 0), (1, 0)]):
        p = new_proposal(4000 + c, U32)
        chain(p, [(j, True) for j in range(3)], vid0=700 * c + 1)
        sessions.append(so.Session(proposal_id=p.proposal_id, timestamp=p.timestamp,
                                   expiration_timestamp=p.expiration_timestamp, expected_voters_count=U32,
                                   round=start, total=0, yes=0, max_rounds=mr, consensus_threshold=T23,
                                   state=po.SESSION_ACTIVE, use_gossipsub_rounds=False, liveness_criteria_yes=True))
        for v in p.votes:
            votes.append(v)
            vs.append(c)
    now = T0 + 5
    ss_ref, out_ref = run_oracle(sessions, votes, vs, now)
    batch, vsess, sarr, owners, osess = device_inputs(sessions, votes, vs)
    st, tr, ins, rs = engine.process_votes(batch, vsess, sarr, owners, osess, now)
    exp = np.array([(o[0], o[1], int(o[2]), o[3]) for o in out_ref], np.int64)
    assert np.array_equal(np.stack([st, tr, ins, rs], axis=1).astype(np.int64), exp)
    assert np.array_equal(sarr, sessions_array(ss_ref))
    assert [int(r) for r in sarr["round"]] == [U32, U32, U32 - 1, 4]
    assert [s.state for s in ss_ref][:2] == [po.SESSION_ACTIVE] * 2 and ss_ref[2].state == po.SESSION_FAILED
