"""Random Proposal messages and byte-level mutations for the wire-decode tests."""
from __future__ import annotations

import random

from hashgraph_like_consensus.protos import Proposal, Vote


def _rbytes(rnd: random.Random, choices) -> bytes:
    n = rnd.choice(choices)
    return bytes(rnd.randrange(256) for _ in range(n))


def random_vote(rnd: random.Random) -> Vote:
    return Vote(
        vote_id=rnd.choice([0, 1, 300, 2**31 + 5, 2**32 - 1, rnd.randrange(2**32)]),
        vote_owner=_rbytes(rnd, [0, 20, 20, 20, 3]),
        proposal_id=rnd.choice([0, 7, 2**32 - 1, rnd.randrange(2**32)]),
        timestamp=rnd.choice([0, 1, 1_760_000_001, 2**64 - 1, rnd.randrange(2**40)]),
        vote=rnd.random() < 0.5,
        parent_hash=_rbytes(rnd, [0, 0, 32]),
        received_hash=_rbytes(rnd, [0, 32, 32]),
        vote_hash=_rbytes(rnd, [0, 32, 32, 32, 200]),
        signature=_rbytes(rnd, [0, 65, 65, 65, 64]),
    )


def random_proposal(rnd: random.Random, max_votes: int = 6) -> Proposal:
    names = ["", "p", "proposal-é中\U0001f600", "x" * 130]
    return Proposal(
        name=rnd.choice(names),
        payload=_rbytes(rnd, [0, 5, 140]),
        proposal_id=rnd.choice([0, 1, 2**32 - 1, rnd.randrange(2**32)]),
        proposal_owner=_rbytes(rnd, [0, 20]),
        votes=[random_vote(rnd) for _ in range(rnd.randrange(max_votes + 1))],
        expected_voters_count=rnd.choice([0, 3, 64, 2**32 - 1]),
        round=rnd.choice([0, 1, 2, 300]),
        timestamp=rnd.choice([0, 1_760_000_000, 2**64 - 1]),
        expiration_timestamp=rnd.choice([0, 1_760_003_600, 2**63]),
        liveness_criteria_yes=rnd.random() < 0.5,
    )


_SPECIAL = [0x00, 0x01, 0x02, 0x07, 0x52, 0x60, 0x72, 0x78, 0x7f, 0x80, 0xff, 0xa0, 0xaa, 0xe2,
            0xfb, 0xfc, 0xc3, 0xed]
_UNKNOWN = [b"\xf8\x01\x05", b"\xf9\x01" + b"\x00" * 8, b"\xfd\x01\x00\x00\x00\x00",
            b"\xfa\x01\x03abc", b"\xfb\x01\x08\x01\xfc\x01", b"\xa8\x03\x01"]


def mutate(rnd: random.Random, msg: bytes) -> bytes:
    b = bytearray(msg)
    for _ in range(rnd.choice([0, 1, 1, 1, 2, 3])):
        op = rnd.randrange(7)
        pos = rnd.randrange(len(b) + 1)
        if op == 0 and b:                      # truncate
            del b[pos:]
        elif op == 1 and pos < len(b):         # flip a bit
            b[pos] ^= 1 << rnd.randrange(8)
        elif op == 2 and pos < len(b):         # special byte
            b[pos] = rnd.choice(_SPECIAL)
        elif op == 3:                          # insert bytes
            b[pos:pos] = bytes(rnd.choice(_SPECIAL) for _ in range(rnd.randrange(1, 4)))
        elif op == 4:                          # splice an unknown field in
            b[pos:pos] = rnd.choice(_UNKNOWN)
        elif op == 5 and pos < len(b):         # delete a byte
            del b[pos]
        elif op == 6 and b:                    # duplicate a segment
            q = rnd.randrange(len(b))
            b[pos:pos] = b[q:q + rnd.randrange(1, 12)]
    return bytes(b)
