"""Pin the oracle (CPU restatements) before trusting it.

The reference ships no byte-level golden vectors, so the oracle is pinned
by published known-answer tests of the third-party algorithms it restates, by independent
implementations that must agree (Python <-> C), and by the protobuf runtime for the encoding.
"""
import hashlib
import random

import numpy as np
import pytest

import coracle
import pyoracle as po

# ---- published KATs --------------------------------------------------------------------
KECCAK_KATS = {
    b"": "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470",
    b"abc": "4e03657aea45a94fc7d47ba826c8d667c0d1e6e33a64a036ec44f58fa12d6c45",
}
# web3.js `eth.accounts.sign("Some data", key)` documentation vector (EIP-191 + RFC 6979 + low-s)
WEB3_KEY = 0x4C0883A69102937D6231471B5DBB6204FE5129617082792AE468D01A3F362318
WEB3_ADDR = "2c7536e3605d9c16a7a3d7b1898e529396a65c23"
WEB3_MSG_HASH = "1da44b586eb0729ff70a73c326926f6ed5a25f5b056e7f47fbc6e58d86871655"
WEB3_SIG = ("b91467e570a6466aa9e9876cbcd013baba02900b8979d43fe208a4a4f339f5fd"
            "6007e74cd82e037b800186422fc2da167c747ef045e5d18a5f5d4300f8e1a0291c")
KEY1_ADDR = "7e5f4552091a69125d5dfcb7b8c2659029395bdf"  # private key 1


@pytest.mark.parametrize("msg,digest", list(KECCAK_KATS.items()))
def test_keccak_kats(msg, digest):
    assert po.keccak256(msg).hex() == digest
    assert coracle.keccak256(msg).hex() == digest


def test_keccak_permutation_matches_hashlib_sha3():
    # same keccak-f[1600], FIPS-202 padding: pins the permutation across block boundaries
    rnd = random.Random(1)
    for n in list(range(0, 300, 7)) + [135, 136, 137, 271, 272, 273]:
        m = bytes(rnd.randrange(256) for _ in range(n))
        assert po.sha3_256_via_keccak(m) == hashlib.sha3_256(m).digest()


def test_keccak_python_vs_c():
    rnd = random.Random(2)
    for n in [0, 1, 64, 135, 136, 137, 200, 271, 272, 500]:
        m = bytes(rnd.randrange(256) for _ in range(n))
        assert po.keccak256(m) == coracle.keccak256(m)


def test_sha256_c_matches_hashlib():
    rnd = random.Random(3)
    for n in [0, 1, 37, 55, 56, 63, 64, 65, 69, 101, 119, 120, 128, 1000]:
        m = bytes(rnd.randrange(256) for _ in range(n))
        assert coracle.sha256(m) == hashlib.sha256(m).digest()


def test_secp256k1_address_kats():
    assert po.privkey_to_address(1).hex() == KEY1_ADDR
    assert po.privkey_to_address(WEB3_KEY).hex() == WEB3_ADDR
    k = np.frombuffer((1).to_bytes(32, "big"), np.uint8).reshape(1, 32)
    assert coracle.address_batch(k, 1)[0].tobytes().hex() == KEY1_ADDR


def test_eip191_sign_recover_web3_vector():
    h = po.eip191_hash_message(b"Some data")
    assert h.hex() == WEB3_MSG_HASH
    assert coracle.eip191_hash(b"Some data").hex() == WEB3_MSG_HASH
    assert po.sign_message(WEB3_KEY, b"Some data").hex() == WEB3_SIG
    key = np.frombuffer(WEB3_KEY.to_bytes(32, "big"), np.uint8).reshape(1, 32)
    assert coracle.sign_batch(key, np.frombuffer(h, np.uint8).reshape(1, 32), 1)[0].tobytes().hex() == WEB3_SIG
    code, addr = po.ecrecover(h, bytes.fromhex(WEB3_SIG))
    assert code == 0 and addr.hex() == WEB3_ADDR
    code, addr = coracle.ecrecover(h, bytes.fromhex(WEB3_SIG))
    assert code == 0 and addr.hex() == WEB3_ADDR


def test_eip191_length_prefix_digits():
    for n in [0, 9, 10, 99, 100, 999, 1000]:
        m = b"x" * n
        assert po.eip191_message(m).startswith(b"\x19Ethereum Signed Message:\n" + str(n).encode())
        assert po.eip191_hash_message(m) == coracle.eip191_hash(m)


def _mutate(rnd, sig):
    s = bytearray(sig)
    k = rnd.randrange(6)
    if k == 1:
        s[rnd.randrange(64)] ^= 1 << rnd.randrange(8)
    elif k == 2:
        s[64] = rnd.choice([0, 1, 2, 26, 29, 34, 35, 36, 37, 255])
    elif k == 3:
        s[32:64] = (po.N - int.from_bytes(s[32:64], "big")).to_bytes(32, "big")
    elif k == 4:
        s[0:32] = rnd.choice([0, po.N, po.N - 1, 2**256 - 1]).to_bytes(32, "big")
    elif k == 5:
        s[32:64] = rnd.choice([0, po.N, po.N // 2, po.N // 2 + 1, 2**256 - 1]).to_bytes(32, "big")
    return bytes(s)


def test_ecrecover_python_vs_c_adversarial():
    """Two independent restatements (big-int Python, 4x64-limb C) agree on every edge class
    of Appendix C: v parsing, high-s normalisation, scalar range, non-residue r."""
    rnd = random.Random(4)
    classes = set()
    for _ in range(120):
        d = rnd.randrange(1, po.N)
        m = bytes(rnd.randrange(256) for _ in range(rnd.randrange(0, 200)))
        h = po.eip191_hash_message(m)
        sig = _mutate(rnd, po.sign_prehash(d, h))
        a = po.ecrecover(h, sig)
        b = coracle.ecrecover(h, sig)
        assert a == b
        classes.add(a[0])
    assert {0, po.SCHEME_BAD_PARITY, po.SCHEME_SCALAR_RANGE}.issubset(classes)


def test_high_s_is_accepted_and_recovers_same_key():
    d = 0x1234567
    h = po.eip191_hash_message(b"vote")
    sig = bytearray(po.sign_prehash(d, h))
    s = int.from_bytes(sig[32:64], "big")
    sig[32:64] = (po.N - s).to_bytes(32, "big")
    sig[64] = 27 + (28 - sig[64])  # flip parity
    code, addr = po.ecrecover(h, bytes(sig))
    assert code == 0 and addr == po.privkey_to_address(d)


def test_crafted_infinity_signature():
    """Q = infinity: pick k, R = kG, s = z/k  =>  s R - z G = 0 (Appendix C)."""
    h = po.eip191_hash_message(b"crafted")
    z = int.from_bytes(h, "big") % po.N
    k = 0xC0FFEE
    R = po.point_mul(k, po.G)
    r = R[0] % po.N
    s = z * pow(k, -1, po.N) % po.N
    v = 27 + (R[1] & 1)  # a high s is normalised by the verifier itself (s R is unchanged)
    sig = r.to_bytes(32, "big") + s.to_bytes(32, "big") + bytes([v])
    assert po.ecrecover(h, sig)[0] == po.SCHEME_INFINITY
    assert coracle.ecrecover(h, sig)[0] == po.SCHEME_INFINITY


def test_no_curve_point_for_r():
    h = po.eip191_hash_message(b"x")
    # smallest r with x^3 + 7 a non-residue
    r = 1
    while po.decompress(r, False) is not None:
        r += 1
    sig = r.to_bytes(32, "big") + (5).to_bytes(32, "big") + b"\x1b"
    assert po.ecrecover(h, sig)[0] == po.SCHEME_NO_POINT
    assert coracle.ecrecover(h, sig)[0] == po.SCHEME_NO_POINT


# ---- prost encoding cross-checked against the protobuf runtime ------------------------------
def _vote_class():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    F = descriptor_pb2.FieldDescriptorProto
    fdp = descriptor_pb2.FileDescriptorProto(name="hlc_test_vote.proto", package="hlctest", syntax="proto3")
    m = fdp.message_type.add(name="Vote")
    for name, num, typ in [("vote_id", 20, F.TYPE_UINT32), ("vote_owner", 21, F.TYPE_BYTES),
                           ("proposal_id", 22, F.TYPE_UINT32), ("timestamp", 23, F.TYPE_UINT64),
                           ("vote", 24, F.TYPE_BOOL), ("parent_hash", 25, F.TYPE_BYTES),
                           ("received_hash", 26, F.TYPE_BYTES), ("vote_hash", 27, F.TYPE_BYTES),
                           ("signature", 28, F.TYPE_BYTES)]:
        m.field.add(name=name, number=num, type=typ, label=F.LABEL_OPTIONAL)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("hlctest.Vote"))


def test_vote_encoding_matches_protobuf_runtime():
    Vote = _vote_class()
    rnd = random.Random(5)
    for t in range(300):
        kw = dict(
            vote_id=rnd.choice([0, 1, 127, 128, 2**31, 2**32 - 1, rnd.randrange(2**32)]),
            vote_owner=bytes(rnd.randrange(256) for _ in range(rnd.choice([0, 1, 20, 200]))),
            proposal_id=rnd.choice([0, 5, 2**32 - 1, rnd.randrange(2**32)]),
            timestamp=rnd.choice([0, 1, 1_760_000_000, 2**63, 2**64 - 1]),
            vote=rnd.random() < 0.5,
            parent_hash=bytes(rnd.randrange(256) for _ in range(rnd.choice([0, 32, 7]))),
            received_hash=bytes(rnd.randrange(256) for _ in range(rnd.choice([0, 32]))),
            vote_hash=bytes(rnd.randrange(256) for _ in range(rnd.choice([0, 32, 300]))),
        )
        ref = Vote(**kw).SerializeToString(deterministic=True)
        assert po.encode_vote(po.Vote(**kw)) == ref
        from hashgraph_like_consensus.protos import Vote as PV, encode_vote
        assert encode_vote(PV(**kw)) == ref
        # the C restatement encodes the same bytes
        from hashgraph_like_consensus.batch import pack_votes
        assert coracle.encode_vote(pack_votes([PV(**kw)]), 0) == ref


def test_canonical_payload_lengths():
    """Canonical payloads (5-byte varints for id/pid/ts): 79 B for a chain's first NO vote
    (1 keccak block with the EIP-191 prefix), 117 B for a chained YES vote (2 blocks)."""
    base = po.Vote(vote_id=0x80000001, vote_owner=b"\x01" * 20, proposal_id=0x80000002,
                   timestamp=1_760_000_001, vote=False, vote_hash=b"\x02" * 32)
    assert len(po.signed_payload(base)) == 79
    assert len(po.eip191_message(po.signed_payload(base))) <= 135
    chained = po.Vote(**{**base.__dict__, "received_hash": b"\x03" * 32, "vote": True})
    assert len(po.signed_payload(chained)) == 117
    assert len(po.eip191_message(po.signed_payload(chained))) > 136
