"""Behavioural scenarios restated from the reference's own tests, as proposals
that the validate-many path must judge exactly like `ConsensusSession::from_proposal`.

Each scenario = (name, Proposal, ConsensusConfig, now, expected status code).  The expected code
is the error class the cited reference test asserts; tests check it against both CPU
restatements and the GPU.
"""
from __future__ import annotations

import copy
from typing import List, Tuple

import pyoracle as po
from adversarial import c_sign, resign

T0 = 1_760_000_000


def key(i: int) -> int:
    return 0x1000 + 7919 * i


def addr(i: int) -> bytes:
    return po.privkey_to_address(key(i))


def mk_vote(p: po.Proposal, choice: bool, signer: int, now: int, vote_id: int) -> po.Vote:
    """utils.rs:55-98 build_vote with an explicit vote_id and the C signer (fast)."""
    owner = addr(signer)
    parent, received = b"", b""
    if p.votes:
        received = p.votes[-1].vote_hash
        for v in reversed(p.votes):
            if v.vote_owner == owner:
                parent = v.vote_hash
                break
    v = po.Vote(vote_id=vote_id, vote_owner=owner, proposal_id=p.proposal_id, timestamp=now, vote=choice,
                parent_hash=parent, received_hash=received)
    v.vote_hash = po.compute_vote_hash(v)
    v.signature = c_sign(key(signer), v)
    return v


def new_proposal(pid: int, n: int, expiration: int = 120, liveness: bool = True, now: int = T0) -> po.Proposal:
    return po.Proposal(name="Proposal", proposal_id=pid, proposal_owner=addr(0), expected_voters_count=n,
                       round=1, timestamp=now, expiration_timestamp=now + expiration,
                       liveness_criteria_yes=liveness)


def chain(p: po.Proposal, signers_choices, now: int = T0 + 1, vid0: int = 1) -> po.Proposal:
    for k, (s, c) in enumerate(signers_choices):
        p.votes.append(mk_vote(p, c, s, now, vid0 + k))
    return p


def scenarios() -> List[Tuple[str, po.Proposal, po.ConsensusConfig, int, int]]:
    G, P2P = po.ConsensusConfig.gossipsub(), po.ConsensusConfig.p2p()
    now = T0 + 5
    out = []

    # vote_validation_tests.rs:44-82 / vote_tests.rs:26-68: valid chained votes
    p = chain(new_proposal(101, 3), [(1, True), (2, True)])
    out.append(("valid_received_link", p, G, now, po.OK))
    # vote_tests.rs:71-114: parent link, same voter (validate_proposal accepts; dup check rejects)
    p = chain(new_proposal(102, 3), [(1, True), (2, False), (1, True)])
    out.append(("parent_link_same_voter_dup", p, G, now, po.DUPLICATE_VOTE))
    # vote_validation_tests.rs:85-135: wrong key -> InvalidVoteSignature
    p = chain(new_proposal(103, 2), [(1, True), (2, True)])
    p.votes[1].signature = c_sign(key(9), p.votes[1])
    out.append(("wrong_key", p, G, now, po.INVALID_VOTE_SIGNATURE))
    # consensus_service_tests.rs:1020-1064: tampered hash -> InvalidVoteHash
    p = chain(new_proposal(104, 3), [(1, True)])
    p.votes[0].vote_hash = bytes([p.votes[0].vote_hash[0] ^ 1]) + p.votes[0].vote_hash[1:]
    out.append(("tampered_hash", p, G, now, po.INVALID_VOTE_HASH))
    # vote_validation_tests.rs:301-334: 64-byte signature -> SignatureScheme
    p = chain(new_proposal(105, 2), [(1, True)])
    p.votes[0].signature = bytes([7]) * 64
    out.append(("sig_len_64", p, G, now, po.SIGNATURE_SCHEME))
    # vote_validation_tests.rs:199-298: empty owner / hash / signature
    for nm, fld, code in (("empty_owner", "vote_owner", po.EMPTY_VOTE_OWNER),
                          ("empty_hash", "vote_hash", po.EMPTY_VOTE_HASH),
                          ("empty_sig", "signature", po.EMPTY_SIGNATURE)):
        p = chain(new_proposal(106, 2), [(1, True)])
        setattr(p.votes[0], fld, b"")
        out.append((nm, p, G, now, code))
    # vote_validation_tests.rs:138-196: bad received_hash -> ReceivedHashMismatch
    p = chain(new_proposal(107, 3), [(1, True), (2, True)])
    p.votes[1].received_hash = bytes(32)
    resign(p.votes[1], key(2))
    out.append(("bad_received", p, G, now, po.RECEIVED_HASH_MISMATCH))
    # vote_validation_tests.rs:337-377: parent -> other owner -> ParentHashMismatch
    p = chain(new_proposal(108, 3), [(1, True), (2, False)])
    p.votes[1].parent_hash = p.votes[0].vote_hash
    resign(p.votes[1], key(2))
    out.append(("parent_other_owner", p, G, now, po.PARENT_HASH_MISMATCH))
    # consensus_service_tests.rs:1119-1161 / session.rs:622-636: duplicate owner
    p = new_proposal(109, 4)
    p.votes.append(mk_vote(p, True, 1, T0 + 1, 1))
    p.votes.append(mk_vote(po.Proposal(proposal_id=109), False, 1, T0 + 1, 2))  # no links
    out.append(("duplicate_owner", p, G, now, po.DUPLICATE_VOTE))
    # rfc_compliance_tests.rs:926-987: replay (ts < creation)
    p = chain(new_proposal(110, 3), [(1, True)], now=T0 - 10)
    out.append(("replay_old_ts", p, G, now, po.TIMESTAMP_OLDER_THAN_CREATION))
    # consensus_service_tests.rs:1164-1216: vote ts > expiration -> VoteExpired
    p = chain(new_proposal(111, 3), [(1, True)], now=T0 + 500)
    out.append(("vote_after_expiry", p, G, now, po.VOTE_EXPIRED))
    # consensus_service_tests.rs:989-1017: proposal expired
    p = chain(new_proposal(112, 3), [(1, True)])
    out.append(("proposal_expired", p, G, T0 + 10_000, po.PROPOSAL_EXPIRED))
    # rfc_compliance_tests.rs:423-488: Gossipsub batch, 3 votes, n = 5
    p = chain(new_proposal(113, 5), [(0, True), (1, True), (2, True)])
    out.append(("gossipsub_batch_3_of_5", p, G, now, po.OK))
    # rfc_compliance_tests.rs:492-573: P2P batch, 6 votes, n = 9 -> YES
    p = chain(new_proposal(114, 9), [(k, True) for k in range(6)])
    out.append(("p2p_batch_6_of_9", p, P2P, now, po.OK))
    # P2P cap ceil(2n/3) = 6: a 7th vote exceeds it (session.rs:306-344)
    p = chain(new_proposal(115, 9), [(k, True) for k in range(7)])
    out.append(("p2p_over_round_cap", p, P2P, now, po.MAX_ROUNDS_EXCEEDED))
    # more votes than expected voters (session.rs:279-282)
    p = chain(new_proposal(116, 2), [(k, True) for k in range(3)])
    out.append(("more_votes_than_voters", p, G, now, po.MAX_ROUNDS_EXCEEDED))
    # Gossipsub with max_rounds override 1: projected round 2 > 1 (scope_config max_rounds_override)
    p = chain(new_proposal(117, 3), [(1, True)])
    out.append(("gossipsub_override_1", p, po.ConsensusConfig(2 / 3, 1, True, True), now, po.MAX_ROUNDS_EXCEEDED))
    # vote for another proposal id (utils.rs:113-115)
    p = chain(new_proposal(118, 3), [(1, True)])
    p.votes[0].proposal_id = 999
    resign(p.votes[0], key(1))
    out.append(("wrong_proposal_id", p, G, now, po.VOTE_PROPOSAL_ID_MISMATCH))
    # empty vote list: StillActive (session.rs:266-268)
    out.append(("no_votes", new_proposal(119, 3), G, now, po.OK))
    # single vote, n = 1: consensus immediately
    p = chain(new_proposal(120, 1), [(1, False)])
    out.append(("single_voter_no", p, G, now, po.OK))
    # tie with everyone voted, liveness false -> NO
    p = chain(new_proposal(121, 4, liveness=False), [(0, True), (1, True), (2, False), (3, False)])
    out.append(("tie_liveness_false", p, G, now, po.OK))
    # high-s signature is accepted (Appendix C)
    p = chain(new_proposal(122, 3), [(1, True), (2, True)])
    s = bytearray(p.votes[1].signature)
    s[32:64] = (po.N - int.from_bytes(s[32:64], "big")).to_bytes(32, "big")
    s[64] = 55 - s[64]
    p.votes[1].signature = bytes(s)
    out.append(("high_s_accepted", p, G, now, po.OK))
    # v = 0/1 and EIP-155 style v are accepted by alloy's normalize_v
    p = chain(new_proposal(123, 3), [(1, True), (2, True)])
    s = bytearray(p.votes[0].signature)
    s[64] = s[64] - 27
    p.votes[0].signature = bytes(s)
    s = bytearray(p.votes[1].signature)
    s[64] = 49 + (s[64] - 27)  # EIP-155 style v: (v - 35) % 2 is the parity
    p.votes[1].signature = bytes(s)
    out.append(("v_raw_and_eip155", p, G, now, po.OK))
    # non-canonical lengths: 19-byte owner -> scheme id-length error after hash check
    p = new_proposal(124, 3)
    v = po.Vote(vote_id=5, vote_owner=b"\x01" * 19, proposal_id=124, timestamp=T0 + 1, vote=True)
    v.vote_hash = po.compute_vote_hash(v)
    v.signature = c_sign(key(3), v)
    p.votes.append(v)
    out.append(("owner_19_bytes", p, G, now, po.SIGNATURE_SCHEME))
    # long vote_hash (never equal to a SHA-256 digest)
    p = chain(new_proposal(125, 3), [(1, True)])
    p.votes[0].vote_hash = p.votes[0].vote_hash + b"\x00"
    out.append(("vote_hash_33_bytes", p, G, now, po.INVALID_VOTE_HASH))
    # oversize fields (beyond the fused kernel's LDS window: exercised on the general GPU path)
    p = chain(new_proposal(126, 3), [(1, True), (2, True)])
    p.votes[1].parent_hash = bytes(range(256)) + bytes(44)
    resign(p.votes[1], key(2))
    out.append(("long_parent_hash", p, G, now, po.PARENT_HASH_MISMATCH))
    p = new_proposal(127, 3)
    v = po.Vote(vote_id=9, vote_owner=bytes(200), proposal_id=127, timestamp=T0 + 1, vote=True)
    v.vote_hash = po.compute_vote_hash(v)
    v.signature = c_sign(key(4), v)
    p.votes.append(v)
    out.append(("owner_200_bytes", p, G, now, po.SIGNATURE_SCHEME))
    # zero ids / zero timestamp encode as omitted proto3 defaults (pid 0, vote_id 0)
    p = new_proposal(0, 2, now=0)
    p.votes.append(mk_vote(p, True, 1, 0, 0))
    out.append(("proto3_defaults", p, G, 5, po.OK))
    return [(nm, copy.deepcopy(p), cfg, t, code) for nm, p, cfg, t, code in out]
