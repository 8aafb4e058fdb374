"""Batched `handle_consensus_timeout` (service.rs:323-373).

KATs restated from the reference's own timeout tests (tests/consensus_service_tests.rs:303-720,
1219-1281): each case is (state, total, yes, n, threshold, liveness) -> (result or Failed).  The
CPU tests pin the oracle on them; the GPU tests run hlc_consensus_timeout_batch on the KATs, on a
randomized sweep checked against the oracle, and through the host service mirror.
"""
import random

import numpy as np
import pytest

import coracle
import pyoracle as po
from hashgraph_like_consensus import _ffi

T23 = 2.0 / 3.0
A, RN, RY, F = po.SESSION_ACTIVE, po.SESSION_REACHED_NO, po.SESSION_REACHED_YES, po.SESSION_FAILED
INSUF = po.INSUFFICIENT_VOTES_AT_TIMEOUT

# (name, state, total, yes, n, t, liveness, expected state, expected status)
KATS = [
    ("already_reached_n2", RY, 2, 2, 2, T23, True, RY, po.OK),                    # :303-347
    ("reaches_yes_2_of_3", A, 2, 2, 3, T23, True, RY, po.OK),                     # :350-412
    ("no_with_multiple_votes", A, 3, 1, 4, T23, False, RN, po.OK),                # :415-484
    ("liveness_yes_1_of_4", A, 1, 1, 4, T23, True, RY, po.OK),                    # :487-546
    ("insufficient_tie", A, 2, 2, 4, T23, False, F, INSUF),                       # :549-629
    ("no_votes_liveness_true", A, 0, 0, 3, T23, True, RY, po.OK),                 # :632-674
    ("no_votes_liveness_false", A, 0, 0, 3, T23, False, RN, po.OK),               # :677-720
    ("failed_is_idempotent", F, 2, 2, 4, T23, False, F, INSUF),                   # :1219-1281
    ("n1_silent", A, 0, 0, 1, T23, True, F, INSUF),                               # n <= 2 needs every vote
    ("reached_no_stands", RN, 1, 0, 5, T23, True, RN, po.OK),
]


def _arr(cases):
    a = np.zeros(len(cases), dtype=_ffi.SESSION_TALLY_DTYPE)
    for k, c in enumerate(cases):
        _, st, total, yes, n, t, live = c[:7]
        a[k]["state"], a[k]["total"], a[k]["yes"] = st, total, yes
        a[k]["expected_voters_count"], a[k]["consensus_threshold"] = n, t
        a[k]["liveness_criteria_yes"] = int(live)
    return a


@pytest.mark.parametrize("case", KATS, ids=[c[0] for c in KATS])
def test_oracle_timeout_kats(case):
    _, st, total, yes, n, t, live, exp_state, exp_status = case
    assert po.handle_consensus_timeout(st, total, yes, n, t, live) == (exp_state, exp_status)
    if st not in (RN, RY):  # the C restatement's tally agrees on the undecided ones
        r = coracle.consensus_result(total, yes, n, t, live, True)
        assert (exp_state == F) == (r is None)


def _random_cases(count, seed):
    rnd = random.Random(seed)
    out = []
    for k in range(count):
        n = rnd.choice([1, 2, 3, 4, 5, 9, 10, 64, 100, 1000, rnd.randrange(1, 10**6), 2**32 - 1])
        total = rnd.randrange(0, min(n, 10**6) + 1)
        yes = rnd.randrange(0, total + 1)
        t = rnd.choice([T23, 0.5, 0.75, 0.9, 1.0, 0.0, rnd.random()])
        st = rnd.choice([A, A, A, F, RN, RY])
        out.append((f"r{k}", st, total, yes, n, t, rnd.random() < 0.5))
    return out


@pytest.mark.gpu
def test_gpu_timeout_kats(engine):
    state, status = engine.consensus_timeout_batch(_arr(KATS))
    for k, c in enumerate(KATS):
        assert (int(state[k]), int(status[k])) == (c[7], c[8]), c[0]


@pytest.mark.gpu
def test_gpu_timeout_random_vs_oracle(engine):
    cases = _random_cases(20000, 7)
    state, status = engine.consensus_timeout_batch(_arr(cases))
    for k, c in enumerate(cases):
        exp = po.handle_consensus_timeout(c[1], c[2], c[3], c[4], c[5], c[6])
        assert (int(state[k]), int(status[k])) == exp, c


@pytest.mark.gpu
def test_gpu_service_timeout_mirror(engine):
    """The reference's flow: accept a proposal with votes, time it out twice (idempotent Failed)."""
    from hashgraph_like_consensus import errors
    from hashgraph_like_consensus.service import ConsensusService
    from scenarios import T0, chain, new_proposal
    svc = ConsensusService(engine)
    p = chain(new_proposal(501, 4, liveness=False), [(1, True), (2, True)])   # 2 YES + 2 silent NO: tie
    q = chain(new_proposal(502, 4, liveness=True), [(1, True)])               # silent count as YES
    svc.process_incoming_proposals("scope", [p, q], T0 + 5)
    res = svc.handle_consensus_timeouts("scope", [501, 502, 999], T0 + 60)
    assert isinstance(res[0], errors.InsufficientVotesAtTimeout)
    assert res[1] is True
    assert isinstance(res[2], errors.SessionNotFound)
    with pytest.raises(errors.InsufficientVotesAtTimeout):
        svc.handle_consensus_timeout("scope", 501, T0 + 61)
    assert svc.handle_consensus_timeout("scope", 502, T0 + 61) is True
