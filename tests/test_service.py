"""The host-side mirror of the reference API (service.py / signing.py / errors.py).

CPU tests drive `ConsensusService` with `OracleEngine`, a test double whose batch calls are the
oracle's (test infrastructure, never shipped): they check config resolution, ProposalAlreadyExist
handling and status -> ConsensusError mapping.  The GPU tests repeat the reference's own
service-level scenarios (tests/rfc_compliance_tests.rs:423-575, consensus_service_tests.rs:886-1020)
through the real libhlc.so path.
"""
from __future__ import annotations

import numpy as np
import pytest

import coracle
from hashgraph_like_consensus import errors
from hashgraph_like_consensus.protos import Proposal, Vote, encode_vote
from hashgraph_like_consensus.service import (ConsensusConfig, ConsensusService, build_vote, resolve_config,
                                              validate_proposals)

T0 = 1_760_000_000


class OracleEngine:
    """Test double with Engine's batch signatures, computed by the oracle."""

    def validate_proposals(self, batch, desc, now, want_votes=True, want_recovered=False):
        return coracle.validate_proposals(batch, desc, now, threads=4)

    def compute_vote_hashes(self, batch):
        return coracle.compute_vote_hashes(batch)

    def process_votes(self, batch, vote_session, sessions, owners=None, owner_session=None, now=0):
        """hlc_process_votes semantics through oracle/stream_oracle.py (sessions updated in place)."""
        import stream_oracle as so
        from adversarial import batch_to_votes
        ss = [so.Session(int(x["proposal_id"]), int(x["timestamp"]), int(x["expiration_timestamp"]),
                         int(x["expected_voters_count"]), int(x["round"]), int(x["total"]), int(x["yes"]),
                         int(x["max_rounds"]), float(x["consensus_threshold"]), int(x["state"]),
                         bool(x["use_gossipsub_rounds"]), bool(x["liveness_criteria_yes"])) for x in sessions]
        for o, k in zip(owners if owners is not None else [], owner_session if owner_session is not None else []):
            ss[int(k)].owners.add(bytes(o))
        out = so.process_incoming_votes(ss, batch_to_votes(batch), [int(v) if v != 0xFFFFFFFF else -1
                                                                    for v in vote_session], now)
        for k, x in enumerate(ss):
            sessions[k]["round"], sessions[k]["total"], sessions[k]["yes"], sessions[k]["state"] = (
                x.round, x.total, x.yes, x.state)
        cols = list(zip(*out)) if out else [(), (), (), ()]
        return tuple(np.array(c, np.uint8) for c in cols)


class OracleSigner:
    """EthereumConsensusSigner's identity/sign over the oracle (test infrastructure)."""

    def __init__(self, seed: int):
        self.key = np.frombuffer(((seed * 0x9E3779B97F4A7C15 + 12345) % (2**255)).to_bytes(32, "big"), np.uint8)
        self.key = self.key.reshape(1, 32).copy()
        self.addr = coracle.address_batch(self.key, 1)[0].tobytes()

    def identity(self):
        return self.addr

    def sign(self, payload: bytes) -> bytes:
        pre = np.frombuffer(coracle.eip191_hash(payload), np.uint8).reshape(1, 32)
        return coracle.sign_batch(self.key, pre, 1)[0].tobytes()


def make_proposal(pid: int, owner, n_votes: int, expected: int, eng, signers=None, now=T0 + 10,
                  expiration=T0 + 3600, yes=True) -> Proposal:
    p = Proposal(name="p", payload=b"x", proposal_id=pid, proposal_owner=owner.identity(), expected_voters_count=expected,
                 timestamp=T0, expiration_timestamp=expiration, liveness_criteria_yes=True)
    signers = signers or [owner] + [OracleSigner(1000 * pid + k) for k in range(1, n_votes)]
    for s in signers[:n_votes]:
        p.votes.append(build_vote(p, yes, s, now, eng))
    return p


# ---------------------------------------------------------------- CPU (oracle-backed double) --
def test_config_presets_and_validation():
    g, p = ConsensusConfig.gossipsub(), ConsensusConfig.p2p()
    assert (g.max_rounds, g.use_gossipsub_rounds) == (2, True)
    assert (p.max_rounds, p.use_gossipsub_rounds) == (0, False)
    assert abs(g.consensus_threshold - 2 / 3) < 1e-15
    with pytest.raises(errors.InvalidConsensusThreshold):
        g.with_threshold(1.5)
    with pytest.raises(errors.InvalidConsensusThreshold):
        g.with_threshold(-0.1)
    with pytest.raises(errors.InvalidTimeout):
        g.with_timeout(0)
    assert g.with_threshold(1.0).consensus_threshold == 1.0


def test_resolve_config_timeout_rule():
    """service.rs:458-466 (and consensus_service_tests.rs:1332): timeout = expiration - timestamp
    only when expiration is after the timestamp."""
    base = ConsensusConfig.gossipsub()
    p = Proposal(timestamp=100, expiration_timestamp=130, liveness_criteria_yes=False)
    c = resolve_config(base, p)
    assert c.consensus_timeout == 30 and c.liveness_criteria is False
    p2 = Proposal(timestamp=100, expiration_timestamp=100, liveness_criteria_yes=True)
    assert resolve_config(base, p2).consensus_timeout == base.consensus_timeout
    assert resolve_config(base, p, explicit=True).consensus_timeout == base.consensus_timeout


def test_error_mapping_covers_every_status():
    for st in list(range(1, 16)):
        e = errors.from_status(st, 3)
        assert isinstance(e, errors.ConsensusError) and e.code == st
    assert isinstance(errors.from_status(7, 5), errors.SignatureScheme)
    assert errors.from_status(7, 5).scheme_error.kind == "Verify"
    with pytest.raises(ValueError):
        errors.from_status(0)


def test_build_vote_chains_like_reference():
    """utils.rs:55-104: received_hash = last vote's hash, parent_hash = own previous vote's hash."""
    eng = OracleEngine()
    a, b = OracleSigner(1), OracleSigner(2)
    p = Proposal(proposal_id=7, expected_voters_count=3, timestamp=T0, expiration_timestamp=T0 + 60)
    v1 = build_vote(p, True, a, T0 + 1, eng)
    assert v1.parent_hash == b"" and v1.received_hash == b""
    p.votes.append(v1)
    v2 = build_vote(p, False, b, T0 + 2, eng)
    assert v2.received_hash == v1.vote_hash and v2.parent_hash == b""
    p.votes.append(v2)
    v3 = build_vote(p, True, a, T0 + 3, eng)
    assert v3.parent_hash == v1.vote_hash and v3.received_hash == v2.vote_hash
    unsigned = Vote(**{**v3.__dict__, "signature": b""})
    pre = coracle.eip191_hash(encode_vote(unsigned))
    rec = coracle.ecrecover(pre, v3.signature)
    assert rec[1] == a.identity()


def test_service_accepts_then_rejects_duplicate_proposal():
    eng = OracleEngine()
    svc = ConsensusService(engine=eng)
    owner = OracleSigner(10)
    p = make_proposal(1, owner, 3, 5, eng)
    svc.process_incoming_proposal("scope", p, T0 + 20)
    rec = svc.get_session("scope", 1)
    assert rec.total == 3 and rec.yes == 3 and rec.config.consensus_timeout == 3600
    with pytest.raises(errors.ProposalAlreadyExist):
        svc.process_incoming_proposal("scope", p, T0 + 20)
    svc.process_incoming_proposal("other", p, T0 + 20)  # scopes are isolated
    with pytest.raises(errors.SessionNotFound):
        svc.get_session("scope", 99)


def test_service_batch_order_semantics():
    """A repeated id in one batch: the first valid copy wins, a copy after an invalid one is
    validated (the reference stores nothing for a rejected proposal)."""
    eng = OracleEngine()
    svc = ConsensusService(engine=eng)
    owner = OracleSigner(11)
    good = make_proposal(5, owner, 2, 4, eng)
    bad = make_proposal(5, owner, 2, 4, eng)
    bad.votes[1] = Vote(**{**bad.votes[1].__dict__, "signature": bytes(65)})
    other = make_proposal(6, owner, 2, 4, eng)
    outs = svc.process_incoming_proposals("s", [bad, good, other, good], T0 + 20)
    assert isinstance(outs[0].error, errors.SignatureScheme)
    assert outs[1].ok and outs[2].ok
    assert isinstance(outs[3].error, errors.ProposalAlreadyExist)
    assert svc.get_session("s", 5).total == 2


def test_service_expired_and_p2p_limits():
    eng = OracleEngine()
    svc = ConsensusService(engine=eng)
    owner = OracleSigner(12)
    p = make_proposal(9, owner, 2, 3, eng, expiration=T0 + 30)
    with pytest.raises(errors.ProposalExpired):
        svc.process_incoming_proposal("s", p, T0 + 31)
    svc.set_scope_config("p2p", ConsensusConfig.p2p())
    p6 = make_proposal(10, owner, 6, 9, eng)          # ceil(2*9/3) = 6 votes allowed
    svc.process_incoming_proposal("p2p", p6, T0 + 20)
    assert svc.get_session("p2p", 10).consensus is True
    p7 = make_proposal(11, owner, 7, 9, eng)
    with pytest.raises(errors.MaxRoundsExceeded):
        svc.process_incoming_proposal("p2p", p7, T0 + 20)


# ---------------------------------------------------------------------------- GPU (libhlc) --
@pytest.mark.gpu
def test_gpu_signer_roundtrip(engine):
    from hashgraph_like_consensus.signing import EthereumConsensusSigner
    s = EthereumConsensusSigner(0x1234567890ABCDEF, engine)
    ref = OracleSigner(0)
    ref.key = np.frombuffer((0x1234567890ABCDEF).to_bytes(32, "big"), np.uint8).reshape(1, 32).copy()
    assert s.identity() == coracle.address_batch(ref.key, 1)[0].tobytes()
    sig = s.sign(b"payload")
    assert sig == ref.sign(b"payload")  # RFC 6979: deterministic
    out = EthereumConsensusSigner.verify_batch([(s.identity(), b"payload", sig),
                                                (s.identity(), b"payloaX", sig),
                                                (s.identity(), b"payload", sig[:64])], engine)
    assert out[0] is True and out[1] is False
    assert isinstance(out[2], errors.ConsensusSchemeError)


@pytest.mark.gpu
def test_gpu_service_matches_oracle_double(engine):
    """Same proposals through the GPU-backed service and the oracle-backed one."""
    eng_o = OracleEngine()
    owner = OracleSigner(21)
    props = [make_proposal(100 + k, owner, 1 + k % 5, 5, eng_o) for k in range(12)]
    props[3].votes[0] = Vote(**{**props[3].votes[0].__dict__, "vote_hash": bytes(32)})
    props[7].votes[-1] = Vote(**{**props[7].votes[-1].__dict__, "timestamp": T0 - 5})
    props.append(props[2])
    a = ConsensusService(engine=engine).process_incoming_proposals("s", props, T0 + 20)
    b = ConsensusService(engine=eng_o).process_incoming_proposals("s", props, T0 + 20)
    for x, y in zip(a, b):
        assert type(x.error) is type(y.error)
        assert (x.transition, x.consensus, x.yes, x.total) == (y.transition, y.consensus, y.yes, y.total)


@pytest.mark.gpu
def test_gpu_reference_batch_scenarios(engine):
    """rfc_compliance_tests.rs:423 (gossipsub batch of 3 accepted) and :492 (p2p batch of 6 of 9
    accepted, consensus YES), consensus_service_tests.rs:886 (duplicate) and :989 (expired)."""
    svc = ConsensusService(engine=engine)
    owner = OracleSigner(31)
    p = make_proposal(1, owner, 3, 5, engine)
    svc.process_incoming_proposal("batch_gossipsub", p, T0 + 20)
    with pytest.raises(errors.ProposalAlreadyExist):
        svc.process_incoming_proposal("batch_gossipsub", p, T0 + 20)
    svc.set_scope_config("batch_p2p", ConsensusConfig.p2p())
    p6 = make_proposal(2, owner, 6, 9, engine)
    svc.process_incoming_proposal("batch_p2p", p6, T0 + 20)
    assert svc.get_session("batch_p2p", 2).consensus is True
    old = make_proposal(3, owner, 1, 3, engine, expiration=T0 + 1)
    with pytest.raises(errors.ProposalExpired):
        svc.process_incoming_proposal("batch_gossipsub", old, T0 + 20)


# ------------------------------------------------ streaming votes (service.rs:286-305) ------------
def _gossip_pair(eng_factory):
    """network_gossip_tests.rs:20-77: peer B stores peer A's vote-less proposal, then receives both
    YES votes of an n = 2 proposal one at a time."""
    eng = eng_factory()
    svc = ConsensusService(engine=eng)
    a, b = OracleSigner(71), OracleSigner(72)
    p = Proposal(name="n2", payload=b"x", proposal_id=4242, proposal_owner=a.identity(), expected_voters_count=2,
                 timestamp=T0, expiration_timestamp=T0 + 3600, liveness_criteria_yes=True)
    svc.process_incoming_proposal("scope", p, T0 + 5)
    va = build_vote(p, True, a, T0 + 6, eng)
    pa = Proposal(**{**p.__dict__, "votes": [va]})
    vb = build_vote(pa, True, b, T0 + 7, eng)
    return svc, va, vb


def _check_gossip(svc, va, vb):
    svc.process_incoming_vote("scope", va, T0 + 8)
    rec = svc.get_session("scope", 4242)
    assert rec.consensus is None and rec.total == 1 and rec.round == 2
    with pytest.raises(errors.DuplicateVote):
        svc.process_incoming_vote("scope", va, T0 + 8)
    svc.process_incoming_vote("scope", vb, T0 + 8)
    assert rec.consensus is True and rec.total == 2 and len(rec.proposal.votes) == 2
    with pytest.raises(errors.SessionNotFound):
        svc.process_incoming_vote("other-scope", va, T0 + 8)
    # a decided session returns its result for further votes without inserting them
    assert svc.process_incoming_votes("scope", [va], T0 + 8) == [None] and rec.total == 2


def test_service_incoming_votes_oracle_double():
    _check_gossip(*_gossip_pair(OracleEngine))


@pytest.mark.gpu
def test_gpu_service_incoming_votes(engine):
    _check_gossip(*_gossip_pair(lambda: engine))


@pytest.mark.gpu
def test_gpu_service_incoming_proposal_bytes(engine):
    """Gossip bytes -> device decode -> validate -> stored session; undecodable bytes and a second
    delivery of the same id get the errors the embedder + reference would produce."""
    from hashgraph_like_consensus.protos import encode_proposal
    svc = ConsensusService(engine=engine)
    owner = OracleSigner(80)
    p = make_proposal(5151, owner, 3, 3, engine)
    msg = encode_proposal(p)
    outs = svc.process_incoming_proposal_bytes("scope", [msg, msg[:-2], msg], T0 + 20)
    assert outs[0].ok and outs[0].total == 3
    assert isinstance(outs[1].error, errors.ProposalDecodeError)
    assert isinstance(outs[2].error, errors.ProposalAlreadyExist)
    rec = svc.get_session("scope", 5151)
    assert rec.proposal == p and rec.owners == {v.vote_owner for v in p.votes}
