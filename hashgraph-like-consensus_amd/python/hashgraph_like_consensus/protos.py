"""Wire types of /root/reference/src/protos/messages/v1/consensus.proto (Proposal 5-16,
Vote 19-29), as plain dataclasses (the reference generates them with prost-build)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List


@dataclass
class Vote:
    vote_id: int = 0              # tag 20, uint32
    vote_owner: bytes = b""       # tag 21
    proposal_id: int = 0          # tag 22, uint32
    timestamp: int = 0            # tag 23, uint64
    vote: bool = False            # tag 24
    parent_hash: bytes = b""      # tag 25
    received_hash: bytes = b""    # tag 26
    vote_hash: bytes = b""        # tag 27
    signature: bytes = b""        # tag 28


@dataclass
class Proposal:
    name: str = ""                       # tag 10
    payload: bytes = b""                 # tag 11
    proposal_id: int = 0                 # tag 12
    proposal_owner: bytes = b""          # tag 13
    votes: List[Vote] = field(default_factory=list)  # tag 14
    expected_voters_count: int = 0       # tag 15
    round: int = 1                       # tag 16
    timestamp: int = 0                   # tag 17
    expiration_timestamp: int = 0        # tag 18
    liveness_criteria_yes: bool = False  # tag 19


def _varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def encode_vote(v: Vote) -> bytes:
    """Host-side proto3 encoding of a Vote (prost `encode_to_vec`), used by the Python
    service layer for small, single-vote calls; the batched GPU path encodes on device."""
    out = bytearray()
    if v.vote_id:
        out += b"\xa0\x01" + _varint(v.vote_id)
    if v.vote_owner:
        out += b"\xaa\x01" + _varint(len(v.vote_owner)) + v.vote_owner
    if v.proposal_id:
        out += b"\xb0\x01" + _varint(v.proposal_id)
    if v.timestamp:
        out += b"\xb8\x01" + _varint(v.timestamp)
    if v.vote:
        out += b"\xc0\x01\x01"
    for key, val in ((b"\xca\x01", v.parent_hash), (b"\xd2\x01", v.received_hash),
                     (b"\xda\x01", v.vote_hash), (b"\xe2\x01", v.signature)):
        if val:
            out += key + _varint(len(val)) + val
    return bytes(out)


def encode_proposal(p: Proposal) -> bytes:
    """prost `encode_to_vec` of a Proposal (consensus.proto:5-16): fields in tag order, proto3
    defaults omitted, each vote a length-delimited tag-14 record (signature included).  The
    wire form the embedder's network layer hands to the device decoder (hlc_decode_proposals)."""
    out = bytearray()
    name = p.name.encode("utf-8") if isinstance(p.name, str) else bytes(p.name)
    if name:
        out += b"\x52" + _varint(len(name)) + name
    if p.payload:
        out += b"\x5a" + _varint(len(p.payload)) + p.payload
    if p.proposal_id:
        out += b"\x60" + _varint(p.proposal_id)
    if p.proposal_owner:
        out += b"\x6a" + _varint(len(p.proposal_owner)) + p.proposal_owner
    for v in p.votes:
        ev = encode_vote(v)
        out += b"\x72" + _varint(len(ev)) + ev
    if p.expected_voters_count:
        out += b"\x78" + _varint(p.expected_voters_count)
    if p.round:
        out += b"\x80\x01" + _varint(p.round)
    if p.timestamp:
        out += b"\x88\x01" + _varint(p.timestamp)
    if p.expiration_timestamp:
        out += b"\x90\x01" + _varint(p.expiration_timestamp)
    if p.liveness_criteria_yes:
        out += b"\x98\x01\x01"
    return bytes(out)
