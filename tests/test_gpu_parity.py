"""GPU parity: libhlc.so (HIP, gfx950) against the CPU restatements, bit-exact.

Every call goes through the C ABI (include/hlc.h) via the product's ctypes engine.
"""
import os
import random

import numpy as np
import pytest

import coracle
import pyoracle as po
from hashgraph_like_consensus import _ffi
from helpers import oracle_workload

pytestmark = pytest.mark.gpu

WEB3_KEY = 0x4C0883A69102937D6231471B5DBB6204FE5129617082792AE468D01A3F362318
WEB3_SIG = bytes.fromhex(
    "b91467e570a6466aa9e9876cbcd013baba02900b8979d43fe208a4a4f339f5fd"
    "6007e74cd82e037b800186422fc2da167c747ef045e5d18a5f5d4300f8e1a0291c")
WEB3_ADDR = bytes.fromhex("2c7536e3605d9c16a7a3d7b1898e529396a65c23")


def _key(d):
    return np.frombuffer(d.to_bytes(32, "big"), np.uint8).reshape(1, 32)


def test_gpu_address_kats(engine):
    keys = np.concatenate([_key(1), _key(WEB3_KEY), _key(po.N - 1), _key(2)])
    addr = engine.address_batch(keys)
    assert addr[0].tobytes().hex() == "7e5f4552091a69125d5dfcb7b8c2659029395bdf"
    assert addr[1].tobytes() == WEB3_ADDR
    assert addr[2].tobytes() == po.privkey_to_address(po.N - 1)
    assert addr[3].tobytes() == po.privkey_to_address(2)


def test_gpu_sign_web3_vector(engine):
    sig = engine.sign_batch(_key(WEB3_KEY), [b"Some data"])
    assert sig[0].tobytes() == WEB3_SIG


def test_gpu_verify_web3_vector(engine):
    st, addr = engine.eth_verify_batch([WEB3_ADDR], [b"Some data"], [WEB3_SIG])
    assert st[0] == 0 and addr[0].tobytes() == WEB3_ADDR


def _mutated_items(n, seed):
    rnd = random.Random(seed)
    ids, pays, sigs = [], [], []
    for t in range(n):
        d = rnd.randrange(1, po.N)
        msg = bytes(rnd.randrange(256) for _ in range(rnd.randrange(0, 300)))
        sig = bytearray(po.sign_message(d, msg) if t < 64 else coracle_sign(d, msg))
        owner = po.privkey_to_address(d) if t < 64 else coracle_addr(d)
        k = rnd.randrange(9)
        if k == 1:
            sig[rnd.randrange(64)] ^= 1 << rnd.randrange(8)
        elif k == 2:
            sig[64] = rnd.choice([0, 1, 2, 26, 29, 34, 35, 36, 37, 255])
        elif k == 3:  # high-s twin: must still be accepted
            s = int.from_bytes(sig[32:64], "big")
            sig[32:64] = (po.N - s).to_bytes(32, "big")
            sig[64] = 27 + (1 - (sig[64] - 27))
        elif k == 4:
            sig[0:32] = rnd.choice([0, po.N, po.N - 1, 2**256 - 1]).to_bytes(32, "big")
        elif k == 5:
            sig[32:64] = rnd.choice([0, po.N, po.N // 2, po.N // 2 + 1, 2**256 - 1]).to_bytes(32, "big")
        elif k == 6:
            owner = bytes(20)
        elif k == 7:
            sig = sig[:rnd.choice([0, 64, 66])] + (b"\x00" if rnd.random() < 0.5 else b"")
        elif k == 8:
            owner = owner[:rnd.choice([0, 19])] + b"\x01" * rnd.choice([0, 2])
        ids.append(bytes(owner))
        pays.append(msg)
        sigs.append(bytes(sig))
    return ids, pays, sigs


def coracle_sign(d, msg):
    h = coracle.eip191_hash(msg)
    return coracle.sign_batch(_key(d), np.frombuffer(h, np.uint8).reshape(1, 32), 1)[0].tobytes()


def coracle_addr(d):
    return coracle.address_batch(_key(d), 1)[0].tobytes()


def _oracle_verify(ids, pays, sigs):
    out_st, out_addr = [], []
    for i, p, s in zip(ids, pays, sigs):
        if len(s) != 65:
            out_st.append(1 + po.SCHEME_SIG_LEN); out_addr.append(bytes(20)); continue
        if len(i) != 20:
            out_st.append(1 + po.SCHEME_ID_LEN); out_addr.append(bytes(20)); continue
        code, addr = coracle.ecrecover(coracle.eip191_hash(p), s)
        if code:
            out_st.append(1 + code); out_addr.append(bytes(20))
        else:
            out_st.append(0 if addr == i else 1); out_addr.append(addr)
    return out_st, out_addr


def test_gpu_verify_batch_adversarial(engine):
    ids, pays, sigs = _mutated_items(1500, 11)
    st, addr = engine.eth_verify_batch(ids, pays, sigs)
    exp_st, exp_addr = _oracle_verify(ids, pays, sigs)
    bad = [i for i in range(len(ids)) if st[i] != exp_st[i] or addr[i].tobytes() != exp_addr[i]]
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}: gpu {[int(st[i]) for i in bad[:5]]} " \
                    f"cpu {[exp_st[i] for i in bad[:5]]}"
    # the mutation mix must exercise every outcome class
    assert {0, 1, 2, 3, 4, 5}.issubset(set(int(x) for x in st))


def test_gpu_vote_hashes_match(engine):
    w = oracle_workload(8, 16, 16, True, 7)
    gpu = engine.compute_vote_hashes(w.batch)
    cpu = coracle.compute_vote_hashes(w.batch)
    assert np.array_equal(gpu, cpu)


def test_gpu_validate_small_workload(engine):
    w = oracle_workload(20, 64, 64, True, 3)
    res, vst, vrs, rec = engine.validate_proposals(w.batch, w.desc, w.now, want_recovered=True)
    cres, cvst, cvrs, crec = coracle.validate_proposals(w.batch, w.desc, w.now, threads=8)
    assert np.array_equal(vst, cvst)
    assert np.array_equal(vrs, cvrs)
    assert np.array_equal(rec, crec)
    assert np.array_equal(res, cres)
    assert (vst == 0).all()


def test_gpu_verify_batch_sizes(engine):
    """k_rec_main hands out 64 votes per wave per grab: batches that are not a multiple of 64,
    smaller than one wave, or end in skipped (pre-rejected) votes must equal the oracle too."""
    ids, pays, sigs = _mutated_items(300, 23)
    exp_st, exp_addr = _oracle_verify(ids, pays, sigs)
    for n in (1, 2, 63, 64, 65, 127, 129, 300):
        st, addr = engine.eth_verify_batch(ids[:n], pays[:n], sigs[:n])
        assert [int(x) for x in st] == exp_st[:n], n
        assert [a.tobytes() for a in addr] == exp_addr[:n], n


@pytest.mark.parametrize("split", ["0", "100", "700", "1", "200,300", "1,1,64"])
def test_gpu_verify_batch_split_schedules(engine, split):
    """hlc_eth_verify_batch stages the items in recovery ranges (HLC_OPT_SPLIT_VOTES: the sizes of the
    ranges before the last), each range's k_rec_prep + k_rec_main behind its upload on two streams in
    turn: every schedule equals the oracle item for item (payloads of 0..299 bytes: 1-3 digit
    EIP-191 lengths, 1-3 keccak blocks)."""
    ids, pays, sigs = _mutated_items(1500, 11)
    exp_st, exp_addr = _oracle_verify(ids, pays, sigs)
    with engine.options(split_votes=split):
        st, addr = engine.eth_verify_batch(ids, pays, sigs)
    assert [int(x) for x in st] == exp_st
    assert [a.tobytes() for a in addr] == exp_addr


def test_gpu_verify_batch_rejects_out_of_arena_outputs_untouched(engine):
    """An item whose (offset, length) leaves the arena: HLC_EINVAL, outputs not written, and the
    context still verifies the next batch."""
    ids, pays, sigs = _mutated_items(300, 5)
    arena = np.frombuffer(b"".join(ids + pays + sigs), np.uint8).copy()
    lens = np.array([len(x) for x in ids + pays + sigs], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))[:-1]]).astype(np.uint64)
    n = len(ids)
    for which, far in ((0, False), (1, False), (2, False), (0, True), (1, True), (2, True)):
        # identity, payload, signature of the last item; far: 2^40, which a kernel would fault on
        o = offs.copy()
        o[which * n + n - 1] = (1 << 40) if far else arena.size + 1
        st = np.full(n, 0xAB, np.uint8)
        addr = np.full((n, 20), 0xAB, np.uint8)
        with engine.options(split_votes=100), pytest.raises(_ffi.HlcError):
            engine.eth_verify_arrays(arena, o[:n], lens[:n], o[n:2 * n], lens[n:2 * n], o[2 * n:], lens[2 * n:],
                                     out=(st, addr))
        assert (st == 0xAB).all() and (addr == 0xAB).all()
    st, addr = engine.eth_verify_arrays(arena, offs[:n], lens[:n], offs[n:2 * n], lens[n:2 * n], offs[2 * n:],
                                        lens[2 * n:])
    assert [int(x) for x in st] == _oracle_verify(ids, pays, sigs)[0]


def test_gpu_verify_large_payloads(engine):
    """hlc_eth_verify_batch hashes each payload in one lane (k_verify_prehash: the EIP-191
    keccak sponge is sequential per message, so one item's latency grows with its length -- about one
    keccak-f per 136 bytes).  Payloads across the block and digit-count boundaries and up to 1 MiB, mixed
    with short ones in one batch, equal the C oracle (its keccak, its recovery) item for item; a flipped
    byte deep inside the 1 MiB payload is a well-formed mismatch (status 1), not an error."""
    rnd = random.Random(77)
    lens = [0, 9, 99, 100, 135, 136, 137, 271, 272, 999, 1000, 4096, 65535, 65536, 1 << 20]
    ids, pays, sigs = [], [], []
    for k, ln in enumerate(lens + [20] * 16):
        d = rnd.randrange(1, po.N)
        msg = rnd.randbytes(ln)
        ids.append(coracle_addr(d))
        pays.append(msg)
        sigs.append(coracle_sign(d, msg))
    big = bytearray(pays[len(lens) - 1])
    big[700_001] ^= 0x40
    ids.append(ids[len(lens) - 1])
    pays.append(bytes(big))
    sigs.append(sigs[len(lens) - 1])
    exp_st, exp_addr = _oracle_verify(ids, pays, sigs)
    st, addr = engine.eth_verify_batch(ids, pays, sigs)
    assert [int(x) for x in st] == exp_st
    assert [a.tobytes() for a in addr] == exp_addr
    assert exp_st[:len(lens)] == [0] * len(lens) and exp_st[-1] == 1
