"""CPU tests of the streaming-vote restatement (oracle/stream_oracle.py) on the reference's own
process_incoming_vote scenarios, plus the ABI layout of hlc_session.

Reference tests mirrored: network_gossip_tests.rs:20-77 (n = 2 needs both YES votes),
81-140 (n = 3, out-of-order delivery converges), consensus_service_tests.rs:919-970 (unknown
session), 1020-1060 (invalid vote hash), rfc_compliance_tests.rs:905-925 (vote on an expired
proposal: VoteExpired or ProposalExpired), plus the add_vote branches of session.rs:225-249.
"""
import os
import subprocess

import pyoracle as po
import stream_oracle as so
from scenarios import T0, mk_vote, new_proposal

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _session(p: po.Proposal, cfg: po.ConsensusConfig = None) -> so.Session:
    cfg = cfg or po.ConsensusConfig.gossipsub()
    return so.Session(proposal_id=p.proposal_id, timestamp=p.timestamp, expiration_timestamp=p.expiration_timestamp,
                      expected_voters_count=p.expected_voters_count, round=1, total=0, yes=0,
                      max_rounds=cfg.max_rounds, consensus_threshold=cfg.consensus_threshold,
                      state=po.SESSION_ACTIVE, use_gossipsub_rounds=cfg.use_gossipsub_rounds,
                      liveness_criteria_yes=p.liveness_criteria_yes)


def _votes(p, signers_choices, now=T0 + 1):
    out = []
    for k, (s, c) in enumerate(signers_choices):
        v = mk_vote(p, c, s, now, 100 + k)
        p.votes.append(v)
        out.append(v)
    return out


def test_two_peers_unanimous_yes_n2():
    p = new_proposal(7, 2)
    va, vb = _votes(p, [(1, True), (2, True)])
    s = [_session(p)]
    out = so.process_incoming_votes(s, [va], [0], T0 + 2)
    assert out == [(po.OK, po.STILL_ACTIVE, True, 0)]
    out = so.process_incoming_votes(s, [vb], [0], T0 + 2)
    assert out == [(po.OK, po.REACHED_YES, True, 0)] and s[0].state == po.SESSION_REACHED_YES


def test_three_peers_out_of_order_converges():
    p = new_proposal(8, 3)
    va, vb = _votes(p, [(1, True), (2, True)])
    for order in ([va, vb], [vb, va]):
        s = [_session(p)]
        out = so.process_incoming_votes(s, order, [0, 0], T0 + 2)
        assert out[-1][:3] == (po.OK, po.REACHED_YES, True) and s[0].total == 2


def test_unknown_session_and_invalid_hash():
    p = new_proposal(9, 3)
    (va,) = _votes(p, [(1, True)])
    s = [_session(p)]
    assert so.process_incoming_votes(s, [va], [-1], T0 + 2)[0][0] == so.SESSION_NOT_FOUND
    bad = po.Vote(**{**va.__dict__})
    bad.vote_hash = bytes(32)
    assert so.process_incoming_votes(s, [bad], [0], T0 + 2)[0][0] == po.INVALID_VOTE_HASH
    assert s[0].total == 0


def test_expired_proposal_vote_rejected():
    p = new_proposal(10, 3, expiration=60)
    (va,) = _votes(p, [(1, True)])
    s = [_session(p)]
    assert so.process_incoming_votes(s, [va], [0], T0 + 61)[0][0] == po.VOTE_EXPIRED          # now > exp
    assert so.process_incoming_votes(s, [va], [0], T0 + 60)[0][0] == po.PROPOSAL_EXPIRED      # now == exp


def test_add_vote_branches():
    p = new_proposal(11, 4)
    va, vb, vc, vd = _votes(p, [(1, True), (2, True), (3, True), (4, False)])
    s = [_session(p)]
    out = so.process_incoming_votes(s, [va, va, vb, vc, vd], [0] * 5, T0 + 2)
    assert out[1][0] == po.DUPLICATE_VOTE
    assert out[3][:3] == (po.OK, po.REACHED_YES, True)
    assert out[4][:3] == (po.OK, po.REACHED_YES, False)          # already decided: not inserted
    s2 = [_session(p)]
    s2[0].state = po.SESSION_FAILED
    assert so.process_incoming_votes(s2, [va], [0], T0 + 2)[0][0] == so.SESSION_NOT_ACTIVE


def test_p2p_round_limit_fails_session():
    p = new_proposal(12, 6)
    vs = _votes(p, [(1, True), (2, False), (3, True), (4, True)])
    s = [_session(p, po.ConsensusConfig(2.0 / 3.0, 2, False, True))]    # P2P, max_rounds 2
    out = so.process_incoming_votes(s, vs, [0] * 4, T0 + 2)
    # round = 1 + votes; the third projects (3 - 1) + 1 = 3 > 2 and fails the session
    assert [o[0] for o in out] == [po.OK, po.OK, po.MAX_ROUNDS_EXCEEDED, so.SESSION_NOT_ACTIVE]
    assert s[0].state == po.SESSION_FAILED and s[0].round == 3 and s[0].total == 2


def test_session_struct_layout(tmp_path):
    from hashgraph_like_consensus import _ffi
    src = tmp_path / "sprobe.c"
    src.write_text(r"""
#include <stdio.h>
#include <stddef.h>
#include "hlc.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(hlc_session),
         offsetof(hlc_session, timestamp), offsetof(hlc_session, expiration_timestamp),
         offsetof(hlc_session, proposal_id), offsetof(hlc_session, expected_voters_count),
         offsetof(hlc_session, round), offsetof(hlc_session, total), offsetof(hlc_session, yes),
         offsetof(hlc_session, max_rounds), offsetof(hlc_session, consensus_threshold),
         offsetof(hlc_session, state), offsetof(hlc_session, use_gossipsub_rounds),
         offsetof(hlc_session, liveness_criteria_yes));
  printf("%d %d\n", HLC_SESSION_NOT_ACTIVE, HLC_SESSION_NOT_FOUND);
  return 0;
}
""")
    exe = tmp_path / "sprobe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    lines = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    vals = list(map(int, lines[0].split()))
    D = _ffi.SESSION_DTYPE
    assert vals == [D.itemsize] + [D.fields[n][1] for n in (
        "timestamp", "expiration_timestamp", "proposal_id", "expected_voters_count", "round", "total", "yes",
        "max_rounds", "consensus_threshold", "state", "use_gossipsub_rounds", "liveness_criteria_yes")]
    assert list(map(int, lines[1].split())) == [so.SESSION_NOT_ACTIVE, so.SESSION_NOT_FOUND]


def test_streaming_workload_builds():
    from stream_cases import run_oracle, streaming_workload
    sessions, votes, vs, now = streaming_workload(0x484C4330, n_props=6, votes=6)
    ss, out = run_oracle(sessions, votes, vs, now)
    codes = {o[0] for o in out}
    assert po.OK in codes and so.SESSION_NOT_FOUND in codes
