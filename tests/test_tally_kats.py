"""Deterministic tally / threshold / round-limit known-answer tests, restated from the reference's
own tests, against both CPU restatements (the GPU's k_finalize is checked in test_gpu_tally.py)."""
import pytest

import coracle
import pyoracle as po

T23 = 2.0 / 3.0

# tests/threshold_tests.rs:9-38 (has_sufficient_votes)
SUFFICIENT = [
    (1, 1, True), (1, 2, False), (2, 2, True), (1, 3, False), (2, 3, True), (2, 4, False), (3, 4, True),
    (3, 5, False), (4, 5, True), (3, 6, False), (4, 6, True), (66, 100, False), (67, 100, True),
]

# tests/threshold_tests.rs:41-165 (calculate_consensus_result): (total, yes, n, t, liveness, timeout, expected)
RESULTS = [
    (3, 2, 3, T23, False, False, True),    # majority yes
    (3, 1, 3, T23, True, False, False),    # majority no
    (2, 1, 2, T23, True, False, False),    # n <= 2: tie is not unanimous YES
    (2, 1, 2, T23, False, False, False),
    (5, 3, 5, 0.9, True, False, None),     # strict threshold
    (3, 2, 5, 0.5, True, False, True),     # fast threshold
    (1, 1, 2, T23, True, True, None),      # n <= 2 unaffected by timeout
    (2, 2, 4, T23, True, False, None),     # quorum not met
    (2, 2, 4, T23, True, True, True),      # timeout, silent -> YES
    (2, 2, 4, T23, False, True, None),     # timeout, silent -> NO, tie
    (2, 1, 4, T23, True, True, True),
    (3, 1, 4, T23, True, True, None),
]

# tests/rfc_compliance_tests.rs:361-372: P2P round cap ceil(2n/3)
CEIL_TABLE = [(1, 1), (2, 2), (3, 2), (4, 3), (5, 4), (6, 4), (7, 5), (8, 6), (9, 6), (10, 7)]


@pytest.mark.parametrize("total,n,ok", SUFFICIENT)
def test_has_sufficient_votes(total, n, ok):
    assert po.has_sufficient_votes(total, n, T23) == ok
    assert (total >= (n if n <= 2 else coracle.threshold_value(n, T23))) == ok


@pytest.mark.parametrize("total,yes,n,t,live,timeout,exp", RESULTS)
def test_calculate_consensus_result(total, yes, n, t, live, timeout, exp):
    assert po.calculate_consensus_result(total, yes, n, t, live, timeout) == exp
    assert coracle.consensus_result(total, yes, n, t, live, timeout) == exp


@pytest.mark.parametrize("n,cap", CEIL_TABLE)
def test_p2p_round_cap_ceil_two_thirds(n, cap):
    assert po.ConsensusConfig.p2p().max_round_limit(n) == cap
    assert coracle.threshold_value(n, T23) == cap
    assert po.check_round_limit(po.ConsensusConfig.p2p(), n, 1, cap)
    assert not po.check_round_limit(po.ConsensusConfig.p2p(), n, 1, cap + 1)


def test_round_limits_session_rs():
    g = po.ConsensusConfig.gossipsub()
    # session.rs:427-469: gossipsub allows any number of votes in round 2 (<= n)
    assert all(po.check_round_limit(g, 4, 1, k) for k in range(0, 5))
    assert not po.check_round_limit(g, 4, 1, 5)          # more than n
    # session.rs:471-524: p2p, n = 5 -> 4 votes
    p = po.ConsensusConfig.p2p()
    assert po.check_round_limit(p, 5, 1, 4) and not po.check_round_limit(p, 5, 1, 5)
    # session.rs:549-551: explicit max_rounds on a non-gossipsub config
    explicit = po.ConsensusConfig(T23, 7, False, True)
    assert explicit.max_round_limit(100) == 7


def test_threshold_edge_arithmetic():
    # (2n).div_ceil(3) in u32 wraps for n >= 2^31 in a release build; f64 path saturates
    n = 2**32 - 1
    assert po.calculate_threshold_based_value(n, T23) == coracle.threshold_value(n, T23) == 1431655765
    assert po.calculate_threshold_based_value(n, 1.0) == coracle.threshold_value(n, 1.0) == 2**32 - 1
    assert po.calculate_threshold_based_value(10, 0.0) == coracle.threshold_value(10, 0.0) == 0
    for n in [3, 10, 1000, 2**20 + 7]:
        for t in [0.5, 0.75, 0.9, 1.0, T23]:
            assert po.calculate_threshold_based_value(n, t) == coracle.threshold_value(n, t)


U32 = 2**32 - 1


def test_p2p_round_limit_rejects_huge_vote_count():
    """session.rs:644-672 (p2p_round_limit_should_reject_effectively_huge_vote_count): a P2P
    session with expected_voters_count = 1 fed vote_count = u32::MAX + 1 must fail
    check_round_limit -- the usize count is compared with n before any u32 truncation."""
    p2p = po.ConsensusConfig.p2p()
    huge = U32 + 1
    assert not po.check_round_limit(p2p, 1, 1, huge)
    assert not coracle.check_round_limit(False, 0, T23, 1, 1, huge)
    # the same count truncated to u32 would be 0 and pass: the order of the checks matters
    assert po.check_round_limit(p2p, 1, 1, huge & U32) and coracle.check_round_limit(False, 0, T23, 1, 1, 0)


def test_p2p_update_round_saturates_at_u32_max():
    """session.rs:674-699 (p2p_update_round_should_advance_for_max_u32_vote_count): from round 1,
    update_round(u32::MAX) advances to exactly u32::MAX (saturating_add, no wrap)."""
    p2p, g = po.ConsensusConfig.p2p(), po.ConsensusConfig.gossipsub()
    assert po.update_round(p2p, 1, U32) == U32 == coracle.update_round(False, 1, U32)
    assert po.update_round(p2p, U32, 1) == U32 == coracle.update_round(False, U32, 1)
    assert po.update_round(p2p, U32 - 1, 1) == U32 == coracle.update_round(False, U32 - 1, 1)
    assert po.update_round(p2p, 7, 3) == 10 == coracle.update_round(False, 7, 3)
    # Gossipsub: round 1 -> 2 on any votes, stays otherwise (session.rs:352-359)
    for r, k, e in [(1, 0, 1), (1, 1, 2), (1, U32, 2), (2, 5, 2)]:
        assert po.update_round(g, r, k) == e == coracle.update_round(True, r, k)


def test_round_limit_boundaries_agree():
    """check_round_limit at the u32 edges, both restatements: P2P projections saturate
    ((round - 1) + count past u32::MAX stays u32::MAX), the ceil(2n/3) cap wraps for n >= 2^31."""
    cases = [
        # (gossipsub, max_rounds, n, round, vote_count, expected)
        (False, U32, U32, U32, 1, True),          # projected saturates to u32::MAX == limit
        (False, U32, U32, U32, 2, True),
        (False, U32 - 1, U32, U32, 1, False),     # saturated projection above an explicit cap
        (False, 0, U32, 1, 1431655765, True),     # (2n).div_ceil(3) wraps: cap 1431655765
        (False, 0, U32, 1, 1431655766, False),
        (False, 0, 2**31 + 5, 1, 4, True),        # 2n wraps to 10 -> cap 4
        (False, 0, 2**31 + 5, 1, 5, False),
        (False, 0, 1, 0, 1, True),                # round 0: saturating_sub keeps 0
        (True, 2, 4, 1, 0, True), (True, 2, 4, 1, 4, True), (True, 1, 4, 1, 1, False),
        (True, 2, 4, 3, 1, False),                # a round past 2 stays as it is
    ]
    for goss, mr, n, r, k, e in cases:
        cfg = po.ConsensusConfig(T23, mr, goss, True)
        assert po.check_round_limit(cfg, n, r, k) == e, (goss, mr, n, r, k)
        assert coracle.check_round_limit(goss, mr, T23, n, r, k) == e, (goss, mr, n, r, k)
