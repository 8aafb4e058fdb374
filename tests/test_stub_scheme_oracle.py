"""The scheme-generic oracle on the CPU: the reference's StubSigner (tests/custom_scheme_tests.rs:33-74)
restated in pyoracle (stub_verify) and in the C oracle (HLCO_STUB) agree vote for vote and proposal for
proposal, every Byzantine kind of tests/stub_scheme.py has its one expected outcome, and the product's
ConsensusSignatureScheme.verify_batch default equals the oracle's verify.  (The GPU side is
tests/test_gpu_scheme_generic.py.)"""
import numpy as np
import pytest

import coracle
import pyoracle as po
from hashgraph_like_consensus import _ffi
from hashgraph_like_consensus.errors import ConsensusSchemeError
from hashgraph_like_consensus.signing import verdict_codes
from stub_scheme import KINDS, NOW, StubSigner, oracle_outcomes, stub_workload

EXPECT = {
    "forge": (po.INVALID_VOTE_SIGNATURE, 0), "sig_short": (po.INVALID_VOTE_SIGNATURE, 0),
    "id_len": (po.SIGNATURE_SCHEME, po.SCHEME_PLUGIN), "tamper_hash": (po.INVALID_VOTE_HASH, 0),
    "empty_sig": (po.EMPTY_SIGNATURE, 0), "ts_old": (po.TIMESTAMP_OLDER_THAN_CREATION, 0),
    "wrong_pid": (po.VOTE_PROPOSAL_ID_MISMATCH, 0), "bad_received": (po.OK, 0), "duplicate": (po.OK, 0), "": (po.OK, 0),
}


def _c_vs_py(props, batch, desc, now):
    vst_py, outs = oracle_outcomes(props, now)
    cres, cvst, cvrs, _ = coracle.validate_proposals(batch, desc, now, threads=4, scheme="stub")
    assert [tuple(x) for x in zip(cvst.tolist(), cvrs.tolist())] == [tuple(x) for x in vst_py]
    for r, o in zip(cres, outs):
        assert int(r["status"]) == o.status
        assert (int(r["bad_index"]) if int(r["bad_index"]) != 0xFFFFFFFF else -1) == o.bad_index
        assert (int(r["yes"]), int(r["total"]), int(r["transition"])) == (o.yes, o.total, o.transition)
    return cres, cvst, cvrs


@pytest.mark.parametrize("seed", [1, 2])
def test_stub_oracles_agree_on_byzantine_mix(seed):
    props, batch, desc, now, kinds = stub_workload(40, 16, seed, fraction=0.35)
    cres, cvst, cvrs = _c_vs_py(props, batch, desc, now)
    got = {}
    for k, s, r in zip(kinds, cvst.tolist(), cvrs.tolist()):
        got.setdefault(k, set()).add((s, r))
    for k in KINDS + [""]:
        assert got.get(k) == {EXPECT[k]}, (k, got.get(k))
    assert {po.OK, po.SIGNATURE_SCHEME, po.INVALID_VOTE_SIGNATURE} <= set(int(s) for s in cres["status"])
    # chain and duplicate outcomes: proposals whose only Byzantine votes are those kinds
    props, batch, desc, now, kinds = stub_workload(30, 12, seed + 10, fraction=0.1,
                                                   kinds_pool=["bad_received", "duplicate"])
    cres, _, _ = _c_vs_py(props, batch, desc, now)
    assert {po.OK, po.DUPLICATE_VOTE, po.RECEIVED_HASH_MISMATCH} <= set(int(s) for s in cres["status"])


def test_stub_clean_batch_reaches_consensus():
    props, batch, desc, now, _ = stub_workload(6, 5, 9)
    cres, cvst, _ = _c_vs_py(props, batch, desc, now)
    assert (cvst == po.OK).all() and (cres["status"] == po.OK).all()


def test_reference_custom_scheme_cases_on_oracle():
    """custom_scheme_tests.rs:91-136 (three stub voters, YES -> consensus) and :139-178 (a forged
    signature -> InvalidVoteSignature), restated on the oracle's from_proposal / validate_vote."""
    p = po.Proposal(name="stub-proposal", payload=b"payload", proposal_id=77, expected_voters_count=3,
                    timestamp=NOW - 10, expiration_timestamp=NOW + 60, liveness_criteria_yes=True)
    for i, ident in enumerate([bytes([1] * 8), bytes([2] * 8), bytes([3] * 8)]):
        v = po.Vote(vote_id=100 + i, vote_owner=ident, proposal_id=77, timestamp=NOW - 5 + i, vote=True,
                    received_hash=p.votes[-1].vote_hash if p.votes else b"")
        v.vote_hash = po.compute_vote_hash(v)
        v.signature = StubSigner(ident).sign(po.signed_payload(v))
        p.votes.append(v)
    o = po.from_proposal(p, po.ConsensusConfig.gossipsub(), NOW, scheme=po.stub_verify)
    assert (o.status, o.transition, o.yes, o.total) == (po.OK, po.REACHED_YES, 3, 3)
    # the Ethereum scheme rejects the same votes: 8-byte identities, 32-byte signatures
    assert po.from_proposal(p, po.ConsensusConfig.gossipsub(), NOW).status == po.SIGNATURE_SCHEME
    forged = po.Vote(**{**p.votes[1].__dict__})
    forged.signature = bytes(b ^ 0xFF for b in forged.signature)
    assert po.validate_vote(forged, p.expiration_timestamp, p.timestamp, NOW, po.stub_verify) == \
        (po.INVALID_VOTE_SIGNATURE, 0)


def test_default_verify_batch_matches_oracle():
    items = [(bytes([7] * 8), b"payload-a", po.stub_sign(bytes([7] * 8), b"payload-a")),
             (bytes([7] * 8), b"payload-a", po.stub_sign(bytes([7] * 8), b"payload-b")),
             (bytes([7] * 9), b"payload-a", po.stub_sign(bytes([7] * 9), b"payload-a")),
             (b"", b"", b"")]
    res = StubSigner.verify_batch(items)
    assert res[0] is True and res[1] is False
    assert isinstance(res[2], ConsensusSchemeError) and isinstance(res[3], ConsensusSchemeError)
    codes = verdict_codes(res)
    want = []
    for ident, payload, sig in items:
        sub, ok, _ = po.stub_verify(ident, payload, sig)
        want.append(_ffi.VERIFY_ERR if ok is None else (_ffi.VERIFY_TRUE if ok else _ffi.VERIFY_FALSE))
        assert sub in (0, po.SCHEME_PLUGIN)
    assert codes.tolist() == want
    assert _ffi.VERIFY_ERR == 1 + po.SCHEME_PLUGIN
