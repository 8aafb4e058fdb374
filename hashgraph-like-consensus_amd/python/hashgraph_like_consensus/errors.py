"""`ConsensusError` (/root/reference/src/error.rs:11-74) and `ConsensusSchemeError`
(/root/reference/src/signing.rs:77-86) as Python exceptions, plus the HLC_* status mapping."""
from __future__ import annotations


class ConsensusSchemeError(Exception):
    """signing.rs:77-86: `Sign(String)` / `Verify(String)`."""

    def __init__(self, kind: str, message: str):
        super().__init__(f"{kind}: {message}")
        self.kind = kind
        self.message = message


class ConsensusError(Exception):
    """Base class; each subclass is one variant of error.rs."""
    code: int = -1


def _variant(name: str, code: int, doc: str):
    cls = type(name, (ConsensusError,), {"code": code, "__doc__": doc})
    return cls


ProposalExpired = _variant("ProposalExpired", 1, "error.rs:39")
VoteProposalIdMismatch = _variant("VoteProposalIdMismatch", 2, "error.rs:41")
EmptyVoteOwner = _variant("EmptyVoteOwner", 3, "error.rs:33")
EmptyVoteHash = _variant("EmptyVoteHash", 4, "error.rs:37")
EmptySignature = _variant("EmptySignature", 5, "error.rs:25")
InvalidVoteHash = _variant("InvalidVoteHash", 6, "error.rs:35")
InvalidVoteSignature = _variant("InvalidVoteSignature", 8, "error.rs:23")
TimestampOlderThanCreationTime = _variant("TimestampOlderThanCreationTime", 9, "error.rs:49")
VoteExpired = _variant("VoteExpired", 10, "error.rs:31")
ReceivedHashMismatch = _variant("ReceivedHashMismatch", 11, "error.rs:43")
ParentHashMismatch = _variant("ParentHashMismatch", 12, "error.rs:45")
DuplicateVote = _variant("DuplicateVote", 13, "error.rs:27")
MaxRoundsExceeded = _variant("MaxRoundsExceeded", 14, "error.rs:65")
ProposalAlreadyExist = _variant("ProposalAlreadyExist", 15, "error.rs:57")
InsufficientVotesAtTimeout = _variant("InsufficientVotesAtTimeout", 16, "error.rs:64")
InvalidConsensusThreshold = _variant("InvalidConsensusThreshold", 100, "error.rs:13-14")
InvalidTimeout = _variant("InvalidTimeout", 101, "error.rs:15-16")
SessionNotActive = _variant("SessionNotActive", 18, "error.rs:53-54 (HLC_SESSION_NOT_ACTIVE)")
SessionNotFound = _variant("SessionNotFound", 19, "error.rs:55-56 (HLC_SESSION_NOT_FOUND)")
ProposalDecodeError = _variant("ProposalDecodeError", 17, "prost DecodeError on the wire bytes (HLC_PROPOSAL_DECODE_ERROR)")


class SignatureScheme(ConsensusError):
    """error.rs:72-73: `SignatureScheme(#[from] ConsensusSchemeError)`."""
    code = 7

    def __init__(self, reason: int = 0):
        super().__init__(f"Signature scheme failure: Verify(reason {reason})")
        self.reason = reason
        self.scheme_error = ConsensusSchemeError("Verify", SCHEME_REASONS.get(reason, str(reason)))


SCHEME_REASONS = {
    1: "expected 65-byte signature",
    2: "expected 20-byte address",
    3: "invalid parity (v)",
    4: "r or s out of range",
    5: "r is not the x-coordinate of a curve point",
    6: "recovered key is the identity",
    7: "the signature scheme rejected the input",  # HLC_SCHEME_PLUGIN: a caller-side scheme's Err(Verify)
}

_BY_CODE = {cls.code: cls for cls in (
    ProposalExpired, VoteProposalIdMismatch, EmptyVoteOwner, EmptyVoteHash, EmptySignature, InvalidVoteHash,
    InvalidVoteSignature, TimestampOlderThanCreationTime, VoteExpired, ReceivedHashMismatch, ParentHashMismatch,
    DuplicateVote, MaxRoundsExceeded, ProposalAlreadyExist, InsufficientVotesAtTimeout, ProposalDecodeError,
    SessionNotActive, SessionNotFound)}


def from_status(status: int, reason: int = 0) -> ConsensusError:
    """HLC_* status code (include/hlc.h) -> the ConsensusError instance the reference returns."""
    if status == SignatureScheme.code:
        return SignatureScheme(reason)
    cls = _BY_CODE.get(status)
    if cls is None:
        raise ValueError(f"not an error status: {status}")
    return cls()
