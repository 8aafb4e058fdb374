"""A non-Ethereum signature scheme for the scheme-generic path (test infrastructure).

`StubSigner` restates the scheme of /root/reference/tests/custom_scheme_tests.rs:33-74, the reference's
proof that `ConsensusService` does not bake in Ethereum (service.rs:39-51): 8-byte identities,
signature = SHA256(identity || payload), `verify` raising Err(Verify) for an identity of any other
length and returning Ok(signature == SHA256(identity || payload)) otherwise.  It implements the product's
`ConsensusSignatureScheme` interface, so the service runs it through the *_verdicts entries.

`stub_workload` builds signed stub-scheme proposals exactly as `build_vote` (utils.rs:55-98) does
(received = the previous vote's hash, parent = the voter's own earlier vote), with a seeded share of
Byzantine votes whose kinds each have one expected outcome:
  forge        signature bytes flipped                      [InvalidVoteSignature: Ok(false)]
  sig_short    signature truncated to 31 bytes              [InvalidVoteSignature: Ok(false)]
  id_len       identity of 7 or 20 bytes, hashed + signed   [SignatureScheme: the stub's Err(Verify)]
  tamper_hash  vote_hash byte flipped                       [InvalidVoteHash]
  empty_sig    signature emptied                            [EmptySignature]
  ts_old       timestamp before creation, hashed + signed   [TimestampOlderThanCreationTime]
  wrong_pid    proposal_id changed, hashed + signed         [VoteProposalIdMismatch]
  bad_received received_hash replaced, hashed + signed      [ReceivedHashMismatch]
  duplicate    a second vote by an earlier voter            [DuplicateVote]
"""
from __future__ import annotations

import hashlib
import random
from typing import List, Tuple

import numpy as np

import pyoracle as po
from hashgraph_like_consensus import _ffi
from hashgraph_like_consensus.batch import pack_votes
from hashgraph_like_consensus.errors import ConsensusSchemeError
from hashgraph_like_consensus.signing import ConsensusSignatureScheme

STUB_IDENTITY_LEN = 8
T0 = 1_760_000_000
NOW = T0 + 1800
KINDS = ["forge", "sig_short", "id_len", "tamper_hash", "empty_sig", "ts_old", "wrong_pid", "bad_received",
         "duplicate"]


class StubSigner(ConsensusSignatureScheme):
    """custom_scheme_tests.rs:33-74 restated on the product interface."""

    def __init__(self, identity: bytes):
        assert len(identity) == STUB_IDENTITY_LEN
        self._identity = bytes(identity)

    @staticmethod
    def expected_signature(identity: bytes, payload: bytes) -> bytes:
        return hashlib.sha256(identity + payload).digest()

    def identity(self) -> bytes:
        return self._identity

    def sign(self, payload: bytes) -> bytes:
        return self.expected_signature(self._identity, payload)

    @staticmethod
    def verify(identity: bytes, payload: bytes, signature: bytes) -> bool:
        if len(identity) != STUB_IDENTITY_LEN:
            raise ConsensusSchemeError(
                "Verify", f"stub identity must be {STUB_IDENTITY_LEN} bytes, got {len(identity)}")
        return signature == StubSigner.expected_signature(identity, payload)


def _finish(v: po.Vote, rehash: bool = True) -> None:
    if rehash:
        v.vote_hash = po.compute_vote_hash(v)
    v.signature = b""
    v.signature = po.stub_sign(v.vote_owner, po.signed_payload(v))


def stub_workload(n_props: int, votes_per: int, seed: int, fraction: float = 0.0, expected: int = 0,
                  kinds_pool=None, clean_every: int = 3) -> Tuple[List[po.Proposal], object, np.ndarray, int, List[str]]:
    """-> (po proposals, VoteBatch, PROPOSAL_DTYPE desc, now, per-vote kind or "").  Every
    `clean_every`-th proposal has no Byzantine vote."""
    rnd = random.Random(seed)
    pool = list(kinds_pool or KINDS)
    expected = expected or votes_per
    props: List[po.Proposal] = []
    kinds: List[str] = []
    k = 0
    for p in range(n_props):
        pid = (0x80000000 | rnd.getrandbits(31)) ^ p
        prop = po.Proposal(name="stub-proposal", payload=b"payload", proposal_id=pid, expected_voters_count=expected,
                           timestamp=T0, expiration_timestamp=T0 + 3600, liveness_criteria_yes=True)
        owners = [hashlib.sha256(b"stub" + seed.to_bytes(8, "little") + p.to_bytes(8, "little") +
                                 j.to_bytes(4, "little")).digest()[:STUB_IDENTITY_LEN] for j in range(votes_per)]
        for j in range(votes_per):
            kind = ""
            if fraction and p % clean_every and rnd.random() < fraction:
                kind = pool[k % len(pool)]
                k += 1
            owner = owners[j]
            if kind == "duplicate" and j > 0:
                owner = owners[rnd.randrange(j)]
            elif kind == "duplicate":
                kind = ""
            if kind == "id_len":
                owner = owner[:7] if rnd.random() < 0.5 else hashlib.sha256(owner).digest()[:20]
            # build_vote (utils.rs:55-98): received = last vote's hash, parent = own earlier vote
            received = prop.votes[-1].vote_hash if prop.votes else b""
            parent = b""
            for u in prop.votes:
                if u.vote_owner == owner:
                    parent = u.vote_hash
            v = po.Vote(vote_id=rnd.getrandbits(32) | 1, vote_owner=owner, proposal_id=pid, timestamp=T0 + 1 + j,
                        vote=rnd.random() < 0.6, parent_hash=parent, received_hash=received)
            if kind == "ts_old":
                v.timestamp = T0 - 5
            elif kind == "wrong_pid":
                v.proposal_id = pid ^ 0x5A5A
            elif kind == "bad_received" and received:
                v.received_hash = hashlib.sha256(received).digest()
            elif kind == "bad_received":
                kind = ""
            _finish(v)
            if kind == "forge":
                v.signature = bytes(b ^ 0xFF for b in v.signature)
            elif kind == "sig_short":
                v.signature = v.signature[:31]
            elif kind == "tamper_hash":
                v.vote_hash = bytes([v.vote_hash[0] ^ 0x01]) + v.vote_hash[1:]
            elif kind == "empty_sig":
                v.signature = b""
            prop.votes.append(v)
            kinds.append(kind)
        props.append(prop)
    batch, desc = pack(props)
    return props, batch, desc, NOW, kinds


def pack(props: List[po.Proposal], config: po.ConsensusConfig = None):
    """po proposals -> (VoteBatch, PROPOSAL_DTYPE desc) under one ConsensusConfig (default gossipsub)."""
    cfg = config or po.ConsensusConfig.gossipsub()
    votes = [v for p in props for v in p.votes]
    desc = np.zeros(len(props), _ffi.PROPOSAL_DTYPE)
    b = 0
    for i, p in enumerate(props):
        desc[i] = (b, len(p.votes), p.proposal_id, p.timestamp, p.expiration_timestamp, p.expected_voters_count,
                   cfg.max_rounds, cfg.consensus_threshold, int(cfg.use_gossipsub_rounds),
                   int(p.liveness_criteria_yes), (0,) * 6)
        b += len(p.votes)
    return pack_votes(votes), desc


def oracle_outcomes(props: List[po.Proposal], now: int, config: po.ConsensusConfig = None):
    """pyoracle under the stub scheme -> (per-vote (status, reason) list, per-proposal outcomes)."""
    cfg = config or po.ConsensusConfig.gossipsub()
    vst = []
    outs = []
    for p in props:
        sts = [po.vote_status_in_proposal(p, v, now, po.stub_verify) for v in p.votes]
        vst.extend(sts)
        outs.append(po.from_proposal(p, cfg, now, vote_status=sts))
    return vst, outs
