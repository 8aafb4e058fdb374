"""CPU tests of the wire-decode oracle (oracle/wire_oracle.py, prost 0.14 `Proposal::decode`
restated) pinned against the protobuf 7.35.1 runtime (upb), and of the host Proposal encoder.

What upb pins: every valid message decodes to the same field values, and whatever upb rejects
the restatement rejects too.  Two classes are prost-only (upb keeps a known field number with the
wrong wire type as an unknown field, where prost returns "invalid wire type"; upb drops the
overflow bits of a 10-byte varint, where prost returns "invalid varint"): there the restatement
follows prost's published source and the result is parity unpinned.
"""
import random

import pytest

import wire_oracle as wo
from hashgraph_like_consensus.protos import Proposal, Vote, encode_proposal
from wire_fuzz import mutate, random_proposal


def _classes():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    F = descriptor_pb2.FieldDescriptorProto
    fdp = descriptor_pb2.FileDescriptorProto(name="hlc_wire_test.proto", package="hlcwire", syntax="proto3")
    p = fdp.message_type.add(name="Proposal")
    for name, num, typ in [("name", 10, F.TYPE_STRING), ("payload", 11, F.TYPE_BYTES),
                           ("proposal_id", 12, F.TYPE_UINT32), ("proposal_owner", 13, F.TYPE_BYTES)]:
        p.field.add(name=name, number=num, type=typ, label=F.LABEL_OPTIONAL)
    p.field.add(name="votes", number=14, type=F.TYPE_MESSAGE, label=F.LABEL_REPEATED, type_name=".hlcwire.Vote")
    for name, num, typ in [("expected_voters_count", 15, F.TYPE_UINT32), ("round", 16, F.TYPE_UINT32),
                           ("timestamp", 17, F.TYPE_UINT64), ("expiration_timestamp", 18, F.TYPE_UINT64),
                           ("liveness_criteria_yes", 19, F.TYPE_BOOL)]:
        p.field.add(name=name, number=num, type=typ, label=F.LABEL_OPTIONAL)
    v = fdp.message_type.add(name="Vote")
    for name, num, typ in [("vote_id", 20, F.TYPE_UINT32), ("vote_owner", 21, F.TYPE_BYTES),
                           ("proposal_id", 22, F.TYPE_UINT32), ("timestamp", 23, F.TYPE_UINT64),
                           ("vote", 24, F.TYPE_BOOL), ("parent_hash", 25, F.TYPE_BYTES),
                           ("received_hash", 26, F.TYPE_BYTES), ("vote_hash", 27, F.TYPE_BYTES),
                           ("signature", 28, F.TYPE_BYTES)]:
        v.field.add(name=name, number=num, type=typ, label=F.LABEL_OPTIONAL)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("hlcwire.Proposal"))


PB = None


def _pb():
    global PB
    if PB is None:
        PB = _classes()
    return PB


VOTE_BYTES = ("vote_owner", "parent_hash", "received_hash", "vote_hash", "signature")


def _agree(msg: bytes, code: int, p) -> None:
    """Compare the restatement's decode of msg with upb's."""
    from google.protobuf.message import DecodeError
    ref = _pb()()
    try:
        ref.ParseFromString(msg)
        upb_ok = True
    except DecodeError:
        upb_ok = False
    if code == wo.OK:
        assert upb_ok, "restatement accepted a message upb rejects"
        sl = lambda t: msg[t[0]:t[0] + t[1]]  # noqa: E731
        assert sl(p.name).decode() == ref.name
        assert sl(p.payload) == ref.payload and sl(p.proposal_owner) == ref.proposal_owner
        assert (p.proposal_id, p.expected_voters_count, p.round, p.timestamp, p.expiration_timestamp,
                p.liveness_criteria_yes) == (ref.proposal_id, ref.expected_voters_count, ref.round,
                                             ref.timestamp, ref.expiration_timestamp, ref.liveness_criteria_yes)
        assert len(p.votes) == len(ref.votes)
        for a, b in zip(p.votes, ref.votes):
            assert (a.vote_id, a.proposal_id, a.timestamp, a.vote) == (b.vote_id, b.proposal_id, b.timestamp, b.vote)
            for f in VOTE_BYTES:
                assert sl(getattr(a, f)) == getattr(b, f)
    elif upb_ok:
        # prost-only rejections (parity unpinned): wrong wire type for a known field, and a
        # 10-byte varint whose last byte overflows u64 (prost checks it, upb drops the bits)
        if code == wo.INVALID_VARINT:
            assert _has_overflowing_varint(msg), "restatement rejects a varint upb accepts"
        else:
            assert code == wo.WIRE_TYPE_MISMATCH, f"restatement rejects ({code}) a message upb accepts"


def _has_overflowing_varint(msg: bytes) -> bool:
    return any(all(b >= 0x80 for b in msg[i:i + 9]) and 2 <= msg[i + 9] < 0x80 for i in range(len(msg) - 9))


def test_encoder_matches_protobuf_runtime():
    rnd = random.Random(11)
    for _ in range(200):
        p = random_proposal(rnd)
        ref = _pb()()
        ref.name = p.name
        ref.payload = p.payload
        ref.proposal_id = p.proposal_id
        ref.proposal_owner = p.proposal_owner
        ref.expected_voters_count = p.expected_voters_count
        ref.round = p.round
        ref.timestamp = p.timestamp
        ref.expiration_timestamp = p.expiration_timestamp
        ref.liveness_criteria_yes = p.liveness_criteria_yes
        for v in p.votes:
            rv = ref.votes.add()
            for f in ("vote_id", "proposal_id", "timestamp", "vote") + VOTE_BYTES:
                setattr(rv, f, getattr(v, f))
        assert encode_proposal(p) == ref.SerializeToString(deterministic=True)


def test_valid_messages_decode_like_upb():
    rnd = random.Random(12)
    for _ in range(300):
        msg = encode_proposal(random_proposal(rnd))
        code, p = wo.decode_proposal(msg)
        assert code == wo.OK
        _agree(msg, code, p)


def test_mutated_messages_agree_with_upb():
    rnd = random.Random(13)
    seen = set()
    for _ in range(3000):
        msg = mutate(rnd, encode_proposal(random_proposal(rnd, max_votes=4)))
        code, p = wo.decode_proposal(msg)
        seen.add(code)
        _agree(msg, code, p)
    # the fuzzer reaches the common error classes
    assert {wo.OK, wo.INVALID_VARINT, wo.BUFFER_UNDERFLOW, wo.WIRE_TYPE_MISMATCH} <= seen


@pytest.mark.parametrize("msg,code", [
    (b"", wo.OK),
    (b"\x60", wo.INVALID_VARINT),                                   # truncated varint
    (b"\x60" + b"\xff" * 9 + b"\x02", wo.INVALID_VARINT),           # 10th byte >= 2
    (b"\x60" + b"\xff" * 9 + b"\x01", wo.OK),                       # 10-byte varint, value truncated to u32
    (b"\x60" + b"\xff" * 10, wo.INVALID_VARINT),                    # 11 bytes
    (b"\x80\x80\x80\x80\x10", wo.INVALID_KEY),                      # key = 2^32
    (b"\x06", wo.INVALID_WIRE_TYPE),                                # key 6: wire type 6 rejected before tag 0
    (b"\x07\x00", wo.INVALID_WIRE_TYPE),
    (b"\x02\x00", wo.INVALID_TAG),                                  # tag 0, wire type 2
    (b"\x61\x00\x00\x00\x00\x00\x00\x00\x00", wo.WIRE_TYPE_MISMATCH),  # proposal_id as fixed64
    (b"\x52\x05abc", wo.BUFFER_UNDERFLOW),
    (b"\x52\x02\xc3\x28", wo.INVALID_UTF8),
    (b"\x52\x03\xed\xa0\x80", wo.INVALID_UTF8),                     # surrogate
    (b"\x72\x03\xa0\x01\x05", wo.OK),                               # one vote with vote_id 5
    (b"\x72\x02\xa0\x01\x05", wo.DELIMITED_EXCEEDED),               # vote field runs past the vote
    (b"\x72\x05\xa0\x01\x05", wo.BUFFER_UNDERFLOW),
    (b"\xfb\x01\x08\x01\xfc\x01", wo.OK),                           # unknown group 31 skipped
    (b"\xfb\x01\x08\x01\x84\x02", wo.UNEXPECTED_END_GROUP),         # mismatched end group
    (b"\xfc\x01", wo.UNEXPECTED_END_GROUP),
    (b"\xf9\x01\x00\x00\x00", wo.BUFFER_UNDERFLOW),                 # unknown fixed64 truncated
])
def test_decode_edge_cases(msg, code):
    got, p = wo.decode_proposal(msg)
    assert got == code
    _agree(msg, got, p)


def test_last_wins_and_repeated_votes():
    v1 = encode_proposal(Proposal(votes=[Vote(vote_id=1)]))
    msg = b"\x60\x05" + b"\x60\x07" + v1 + v1 + b"\x52\x01a\x52\x01b"
    code, p = wo.decode_proposal(msg)
    assert code == wo.OK and p.proposal_id == 7 and len(p.votes) == 2 and msg[p.name[0]] == ord("b")
    _agree(msg, code, p)


def test_workload_wire_encoding_roundtrips():
    """synth.to_wire (the wire form bench.py and the GPU tests feed the device decoder) decodes,
    under the restated prost decoder, back to exactly the SoA workload it came from."""
    import numpy as np
    from hashgraph_like_consensus import synth
    from helpers import oracle_workload

    w = oracle_workload(3, 5, 8, True, 0x484C4320, name="wire-rt")
    wire, off, lens, scope = synth.to_wire(w.batch, w.desc)
    b = w.batch
    for p in range(w.desc.shape[0]):
        msg = wire[int(off[p]):int(off[p]) + int(lens[p])].tobytes()
        code, dp = wo.decode_proposal(msg)
        d = w.desc[p]
        assert code == wo.OK and len(dp.votes) == int(d["vote_count"])
        assert (dp.proposal_id, dp.timestamp, dp.expiration_timestamp, dp.expected_voters_count,
                dp.liveness_criteria_yes) == (int(d["proposal_id"]), int(d["timestamp"]),
                                              int(d["expiration_timestamp"]), int(d["expected_voters_count"]),
                                              bool(d["liveness_criteria_yes"]))
        assert scope[p]["max_rounds"] == d["max_rounds"] and scope[p]["use_gossipsub_rounds"] == d["use_gossipsub_rounds"]
        for j, v in enumerate(dp.votes):
            i = int(d["vote_begin"]) + j
            assert (v.vote_id, v.proposal_id, v.timestamp, v.vote) == (
                int(b.vote_id[i]), int(b.proposal_id[i]), int(b.timestamp[i]), bool(b.vote[i]))
            for k, f in enumerate(("vote_owner", "parent_hash", "received_hash", "vote_hash", "signature")):
                o, ln = getattr(v, f)
                assert msg[o:o + ln] == b.field(i, k)
    assert np.array_equal(scope["consensus_threshold"], w.desc["consensus_threshold"])
