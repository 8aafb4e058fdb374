"""GPU parity of the wire path (hlc_wire.hip through the C ABI) against the oracles.

  * decode: fuzzed Proposal messages (valid, and mutated into every prost DecodeError class)
    decoded on the device == oracle/wire_oracle.py (prost 0.14 restated): status, failing
    record, every scalar and every (offset, length) of every vote;
  * validate from wire: hlc_validate_wire_proposals on encoded workloads (clean, Byzantine, and
    with undecodable messages mixed in) == the C oracle's from_proposal outcomes on the same
    proposals, and == the SoA path (hlc_validate_proposals) -- bit for bit.
"""
import os
import random

import numpy as np
import pytest

import coracle
import wire_oracle as wo
from adversarial import byzantine
from hashgraph_like_consensus import _ffi, synth
from hashgraph_like_consensus.protos import encode_proposal
from helpers import oracle_workload
from wire_fuzz import mutate, random_proposal

pytestmark = pytest.mark.gpu
THREADS = max(1, min(16, os.cpu_count() or 1))
VOTE_FIELDS = ("vote_owner", "parent_hash", "received_hash", "vote_hash", "signature")


def _pack(msgs):
    lens = np.array([len(m) for m in msgs], np.uint32)
    off = np.zeros(len(msgs), np.uint64)
    if msgs:
        off[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
    return np.frombuffer(b"".join(msgs) or b"\0", np.uint8)[:int(lens.sum())].copy(), off, lens


def _scope(n, gossipsub=True):
    sc = np.zeros(n, _ffi.SCOPE_CONFIG_DTYPE)
    sc["consensus_threshold"] = 2.0 / 3.0
    sc["max_rounds"] = 2 if gossipsub else 0
    sc["use_gossipsub_rounds"] = 1 if gossipsub else 0
    return sc


def _check_decode(engine, msgs, scope):
    wire, off, lens = _pack(msgs)
    props, winfo, batch = engine.decode_proposals(wire, off, lens, scope)
    codes = set()
    for m, msg in enumerate(msgs):
        code, p, bad = wo.decode_proposal_ex(msg)
        codes.add(code)
        w = winfo[m]
        assert int(w["decode_status"]) == code, f"message {m}: status {int(w['decode_status'])} != {code}"
        assert int(w["bad_vote"]) == bad, f"message {m}: bad vote"
        d = props[m]
        sc = scope[0] if scope.shape[0] == 1 else scope[m]
        assert d["max_rounds"] == sc["max_rounds"] and d["use_gossipsub_rounds"] == sc["use_gossipsub_rounds"]
        assert d["consensus_threshold"] == sc["consensus_threshold"]
        if code != wo.OK:
            assert int(d["vote_count"]) == 0
            continue
        assert (int(d["proposal_id"]), int(d["timestamp"]), int(d["expiration_timestamp"]),
                int(d["expected_voters_count"]), bool(d["liveness_criteria_yes"])) == (
            p.proposal_id, p.timestamp, p.expiration_timestamp, p.expected_voters_count, p.liveness_criteria_yes)
        assert int(w["round"]) == p.round
        for k, f in (("name", "name"), ("payload", "payload"), ("owner", "proposal_owner")):
            assert (int(w[f"{k}_off"]), int(w[f"{k}_len"])) == getattr(p, f), f"message {m}: {f}"
        assert int(d["vote_count"]) == len(p.votes)
        base = int(off[m])
        for j, v in enumerate(p.votes):
            i = int(d["vote_begin"]) + j
            assert (int(batch.vote_id[i]), int(batch.proposal_id[i]), int(batch.timestamp[i]),
                    bool(batch.vote[i])) == (v.vote_id, v.proposal_id, v.timestamp, v.vote), f"msg {m} vote {j}"
            for k, f in enumerate(VOTE_FIELDS):
                o, ln = getattr(v, f)
                assert int(batch.field_len[i, k]) == ln, f"msg {m} vote {j} {f} length"
                if ln:
                    assert int(batch.field_off[i, k]) == base + o, f"msg {m} vote {j} {f} offset"
    return codes


def test_gpu_decode_fuzzed_messages(engine):
    rnd = random.Random(21)
    msgs = []
    for t in range(1500):
        msg = encode_proposal(random_proposal(rnd, max_votes=5))
        msgs.append(msg if t % 3 == 0 else mutate(rnd, msg))
    # hand-made edge cases: empty message, groups, deep group nesting, UTF-8, delimited overrun
    msgs += [b"", b"\xfb\x01\x08\x01\xfc\x01", b"\xfb\x01" * 120 + b"\xfc\x01" * 120,
             b"\xfb\x01" * 99 + b"\xfc\x01" * 99, b"\x72\x08\xfb\x01" * 1 + b"\xfb\x01\xfc\x01\xfc\x01\x00\x00",
             b"\x52\x03\xed\xa0\x80", b"\x52\x04\xf0\x9f\x98\x80", b"\x72\x02\xa0\x01\x05",
             b"\x60" + b"\xff" * 9 + b"\x01", b"\x60" + b"\xff" * 9 + b"\x02"]
    codes = _check_decode(engine, msgs, _scope(1))
    assert {wo.OK, wo.INVALID_VARINT, wo.BUFFER_UNDERFLOW, wo.WIRE_TYPE_MISMATCH, wo.INVALID_UTF8,
            wo.DELIMITED_EXCEEDED, wo.RECURSION_LIMIT} <= codes


@pytest.mark.parametrize("walker", ["lane", "lds"])
def test_gpu_decode_fuzzed_messages_both_walkers(engine, monkeypatch, walker):
    """Both top-level walkers (HLC_WIRE_WALK: k_wire_walk, one lane per message; k_wire_walk_lds, message
    windows staged in LDS) against the prost restatement: fuzzed messages, messages longer than the LDS
    window (12 KB: the walker reads past it from global memory) and messages at odd byte offsets."""
    from wire_fuzz import random_vote
    from hashgraph_like_consensus.protos import Proposal
    monkeypatch.setenv("HLC_WIRE_WALK", walker)
    rnd = random.Random(24)
    msgs = []
    for t in range(600):
        msg = encode_proposal(random_proposal(rnd, max_votes=5))
        msgs.append(msg if t % 3 == 0 else mutate(rnd, msg))
    for t in range(6):  # 70-110 vote records: past the 12 KB window, some mutated near their end
        big = encode_proposal(Proposal(name="w", proposal_id=70 + t, expected_voters_count=200,
                                       votes=[random_vote(rnd) for _ in range(70 + 8 * t)]))
        msgs.append(big if t % 2 == 0 else big[:-3] + bytes([rnd.randrange(256)]) + big[-2:])
    msgs.insert(7, b"\x01")  # every later message starts at an odd offset
    codes = _check_decode(engine, msgs, _scope(1))
    assert {wo.OK, wo.INVALID_VARINT, wo.BUFFER_UNDERFLOW, wo.WIRE_TYPE_MISMATCH} <= codes


def test_gpu_decode_per_message_scope_and_overlap(engine):
    rnd = random.Random(22)
    msgs = [encode_proposal(random_proposal(rnd, max_votes=3)) for _ in range(40)]
    sc = _scope(40)
    sc["max_rounds"] = np.arange(40)
    sc["use_gossipsub_rounds"] = np.arange(40) % 2
    _check_decode(engine, msgs, sc)
    # the same bytes referenced by two messages
    wire, off, lens = _pack(msgs[:1])
    props, winfo, batch = engine.decode_proposals(wire, np.array([0, 0], np.uint64), np.array([lens[0]] * 2, np.uint32),
                                                  _scope(1))
    assert props[0]["vote_count"] == props[1]["vote_count"] and batch.n == 2 * int(props[0]["vote_count"])


def test_gpu_decode_empty_and_capacity(engine):
    props, winfo, batch = engine.decode_proposals(b"", np.zeros(0, np.uint64), np.zeros(0, np.uint32), _scope(1))
    assert props.shape[0] == 0 and batch.n == 0


def _wire_vs_oracle(engine, w_batch, desc, now, extra_msgs=()):
    wire, off, lens, scope = synth.to_wire(w_batch, desc)
    if extra_msgs:  # undecodable messages appended (decode errors must not disturb the rest)
        ew, eo, el = _pack(list(extra_msgs))
        off = np.concatenate([off, eo + np.uint64(wire.size)])
        lens = np.concatenate([lens, el])
        wire = np.concatenate([wire, ew])
        scope = np.concatenate([scope, _scope(len(extra_msgs))])
    res, winfo, nv = engine.validate_wire_proposals(wire, off, lens, scope, now)
    P = desc.shape[0]
    # vote records walked (those of messages that fail later included), as hlc_decode_proposals counts them
    props, _, dbatch = engine.decode_proposals(wire, off, lens, scope)
    assert nv == dbatch.n and (props["vote_count"][:P] == desc["vote_count"]).all()
    assert (winfo["decode_status"][:P] == 0).all()
    cres, _, _, _ = coracle.validate_proposals(w_batch, desc, now, threads=THREADS)
    bad = np.nonzero(res[:P] != cres)[0]
    assert bad.size == 0, f"{bad.size} proposals differ from the oracle, first {bad[:5]}: {res[bad[:3]]} vs {cres[bad[:3]]}"
    sres, _, _, _ = engine.validate_proposals(w_batch, desc, now, want_votes=False)
    assert np.array_equal(res[:P], sres)
    for k, m in enumerate(extra_msgs):
        code, p, badv = wo.decode_proposal_ex(m)
        r = res[P + k]
        if code == wo.OK:
            continue
        assert (int(r["status"]), int(r["scheme_reason"]), int(r["bad_index"])) == (
            17, code, badv)  # HLC_PROPOSAL_DECODE_ERROR
    return res


def test_gpu_validate_wire_clean_and_decode_errors(engine):
    w = oracle_workload(24, 16, 16, True, 0x484C4311, name="wire-clean")
    rnd = random.Random(23)
    extra = [mutate(rnd, encode_proposal(random_proposal(rnd, max_votes=3))) for _ in range(60)]
    res = _wire_vs_oracle(engine, w.batch, w.desc, w.now, extra)
    assert (res["status"][:24] == 0).all()


def test_gpu_validate_wire_byzantine(engine):
    w = oracle_workload(48, 16, 16, True, 0x484C4312, name="wire-byz")
    batch, desc, kinds = byzantine(w, fraction=1 / 3, seed=7)
    res = _wire_vs_oracle(engine, batch, desc, w.now)
    assert (res["status"] != 0).sum() > 0


def test_gpu_validate_wire_p2p(engine):
    w = oracle_workload(6, 40, 60, False, 0x484C4313, name="wire-p2p")
    _wire_vs_oracle(engine, w.batch, w.desc, w.now)


def test_gpu_decode_large_messages(engine):
    """Messages with more vote records than the walker keeps per message (128) and spanning many
    4 KiB walker windows, mixed with small ones and a corrupted large one."""
    from wire_fuzz import random_vote
    from hashgraph_like_consensus.protos import Proposal
    rnd = random.Random(24)
    msgs = []
    for k in range(6):
        p = random_proposal(rnd, max_votes=3)
        if k % 2 == 0:
            p = Proposal(name="big", proposal_id=1000 + k, votes=[random_vote(rnd) for _ in range(130 + 70 * k)],
                         expected_voters_count=500, timestamp=5, expiration_timestamp=9)
        msgs.append(encode_proposal(p))
    big = bytearray(msgs[2])
    big[len(big) // 2] ^= 0x80  # corrupt somewhere in the middle of the vote records
    msgs.append(bytes(big))
    _check_decode(engine, msgs, _scope(1))


def test_gpu_decode_capacity_contract(engine):
    """hlc_decode_proposals: too small a vote capacity -> HLC_ERANGE with the needed count reported
    and the proposal records still written; NULL vote arrays query the count."""
    import ctypes
    from ctypes import c_uint8, c_uint32, c_uint64, c_void_p
    rnd = random.Random(25)
    msgs = [encode_proposal(random_proposal(rnd, max_votes=4)) for _ in range(8)]
    wire, off, lens = _pack(msgs)
    sc = _scope(1)
    props = np.zeros(8, _ffi.PROPOSAL_DTYPE)
    nv = c_uint64(0)
    lib = engine.lib
    args = (engine.ctx, _ffi.ptr(wire, c_uint8), wire.size, _ffi.ptr(off, c_uint64), _ffi.ptr(lens, c_uint32), 8,
            c_void_p(sc.ctypes.data), 1, c_void_p(props.ctypes.data), None, ctypes.byref(nv))
    assert lib.hlc_decode_proposals(*args, None, None, None, None, None, None) == 0
    need = nv.value
    assert need == sum(len(wo.decode_proposal(m)[1].votes) for m in msgs)
    if need == 0:
        return
    small = [np.zeros(max(need, 1) * k, dt) for k, dt in ((1, np.uint32), (1, np.uint32), (1, np.uint64),
                                                           (1, np.uint8), (5, np.uint64), (5, np.uint32))]
    nv.value = need - 1
    props[:] = 0
    rc = lib.hlc_decode_proposals(*args, *[_ffi.ptr(a, t) for a, t in zip(small, (c_uint32, c_uint32, c_uint64, c_uint8,
                                                                                 c_uint64, c_uint32))])
    assert rc == -5 and nv.value == need          # HLC_ERANGE, count reported
    assert int(props["vote_count"].sum()) == need  # proposal records written anyway
    assert all(not a.any() for a in small)         # vote arrays untouched


def _hip():
    """The HIP runtime libhlc.so itself uses (already loaded by the engine): device buffers for the
    device-pointer entry points without a second runtime in the process."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    return hip


def test_gpu_wire_device_entry_misaligned(engine):
    """hlc_validate_wire_proposals_device on a wire pointer that is not 16-byte aligned (the
    walker's and vote kernel's byte-wise fallback paths) == the host-buffer entry."""
    import ctypes
    from ctypes import c_void_p
    hip = _hip()
    w = oracle_workload(6, 8, 8, True, 0x484C4314, name="wire-misaligned")
    wire, off, lens, scope = synth.to_wire(w.batch, w.desc)
    ref, rw, _ = engine.validate_wire_proposals(wire, off, lens, scope, w.now)
    m = off.size

    def dev(nbytes):
        p = c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), max(nbytes, 16)) == 0
        return p

    def h2d(d, a):
        assert hip.hipMemcpy(d, a.ctypes.data, a.nbytes, 1) == 0

    def d2h(a, d):
        assert hip.hipMemcpy(a.ctypes.data, d, a.nbytes, 2) == 0

    bufs = {k: dev(n) for k, n in (("wire", wire.size + 16), ("off", off.nbytes), ("len", lens.nbytes),
                                    ("scope", scope.nbytes), ("res", m * 16), ("wi", m * 48))}
    try:
        h2d(bufs["off"], off)
        h2d(bufs["len"], lens)
        h2d(bufs["scope"], scope)
        for shift in (0, 3, 8):
            padded = np.zeros(wire.size + 16, np.uint8)
            padded[shift:shift + wire.size] = wire
            h2d(bufs["wire"], padded)
            _ffi.check(engine.lib.hlc_validate_wire_proposals_device(
                engine.ctx, c_void_p(bufs["wire"].value + shift), wire.size, bufs["off"], bufs["len"], m,
                bufs["scope"], scope.size, w.now, bufs["res"], bufs["wi"], None))
            assert hip.hipDeviceSynchronize() == 0  # the entry is asynchronous on the context's stream
            res = np.zeros(m, _ffi.RESULT_DTYPE)
            wi = np.zeros(m, _ffi.WIRE_PROPOSAL_DTYPE)
            d2h(res, bufs["res"])
            d2h(wi, bufs["wi"])
            assert np.array_equal(res, ref), f"shift {shift}: results differ"
            assert np.array_equal(wi, rw), f"shift {shift}: wire info differs"
    finally:
        for p in bufs.values():
            hip.hipFree(p)


def test_gpu_wire_single_large_p2p_proposal(engine):
    """One P2P proposal with 20,000 chained votes as a single gossip message: the walker's second
    pass (> 128 records) and the global chain / duplicate tables (> 512 votes) behind the wire
    path, against the SoA path and the C oracle; plus a re-linked vote and a replayed voter."""
    w = synth.generate(1, 20_000, 30_000, False, synth.config_seed(3), *synth.engine_signers(engine))
    res = _wire_vs_oracle(engine, w.batch, w.desc, w.now)
    assert int(res[0]["status"]) == 0 and int(res[0]["total"]) == 20_000
    # a duplicate voter: vote 15000's owner bytes replaced by vote 100's (hash and signature now
    # fail too, so the first error is that vote's own validation failure, not the chain)
    b = w.batch
    o1, o2 = int(b.field_off[15_000, 0]), int(b.field_off[100, 0])
    b.arena[o1:o1 + 20] = b.arena[o2:o2 + 20]
    res = _wire_vs_oracle(engine, b, w.desc, w.now)
    assert int(res[0]["status"]) != 0 and int(res[0]["bad_index"]) == 15_000


def test_gpu_decode_huge_messages_parallel_path(engine):
    """Messages over 1 MiB (hlc_wire.hip's parallel boundary-discovery path: next[] per byte offset
    + pointer jumping) == the prost oracle, mixed with small (serially walked) messages: a clean
    one, scalars repeated after the votes (last wins), an unknown field, a bad UTF-8 name after the
    votes, a top-level group longer than the bounded per-offset skip, a truncated one, one corrupted mid-records, and one whose huge payload holds no votes."""
    from wire_fuzz import random_vote
    from hashgraph_like_consensus.protos import Proposal
    rnd = random.Random(31)
    votes = [random_vote(rnd) for _ in range(6000)]
    base = encode_proposal(Proposal(name="huge", proposal_id=7, votes=votes, expected_voters_count=9000,
                                    timestamp=5, expiration_timestamp=99, round=2))
    assert len(base) > (1 << 20)
    bad_mid = bytearray(base)
    bad_mid[len(bad_mid) // 2:len(bad_mid) // 2 + 12] = b"\xff" * 12
    msgs = [
        encode_proposal(random_proposal(rnd, max_votes=3)),
        base,
        base + b"\x52\x03abc" + b"\x60\x2a" + b"\x80\x01\x05",   # name, proposal_id again; tag 16 varint
        base + b"\x98\x06\x07",                                  # unknown field 99, varint
        base + b"\x52\x02\xff\xfe",                              # invalid UTF-8 name after the votes
        base[:-5],                                               # truncated
        base + b"\xfb\x01\x0a\x80\x02" + bytes(256) + b"\xfc\x01\x60\x2b",  # top-level group > 256 B, then a scalar
        bytes(bad_mid),
        encode_proposal(random_proposal(rnd, max_votes=2)),
        encode_proposal(Proposal(name="p", payload=bytes(rnd.getrandbits(8) for _ in range(1_200_000)))),
    ]
    _check_decode(engine, msgs, _scope(1))


def test_gpu_decode_huge_message_many_long_groups(engine):
    """Thousands of top-level unknown groups longer than the bounded per-offset skip (256 B) in
    messages over 1 MiB: the chain stops at the first one and a single lane finishes the walk
    (k_huge_tail), linear in the message -- the outcome must equal the prost oracle, including
    votes and scalars after the groups, an unterminated group, and an error after them."""
    from wire_fuzz import random_vote
    from hashgraph_like_consensus.protos import Proposal
    rnd = random.Random(37)
    grp = b"\xfb\x01\x0a\x90\x02" + bytes(272) + b"\xfc\x01"          # group (field 31) holding a 272-B blob
    votes = [random_vote(rnd) for _ in range(300)]
    head = encode_proposal(Proposal(name="g", proposal_id=9, votes=votes[:150], expected_voters_count=400))
    tail = encode_proposal(Proposal(votes=votes[150:], timestamp=11, expiration_timestamp=77))
    many = head + grp * 4000 + tail + b"\x60\x2c"                    # > 1 MiB, 4000 groups, then a scalar
    assert len(many) > (1 << 20)
    msgs = [
        many,
        head + grp * 4000 + b"\xfb\x01\x0a\x02ab",                 # unterminated group at the end
        head + grp * 3000 + b"\x60\xff\xff\xff\xff\xff\xff\xff\xff\xff\xff\x01" + tail,  # bad varint after groups
        encode_proposal(random_proposal(rnd, max_votes=2)),
    ]
    _check_decode(engine, msgs, _scope(1))


def test_gpu_decode_huge_message_long_group_first(engine):
    """a top-level group longer than the bounded per-offset skip at the START of a huge
    message used to hand the whole message to one lane.  The chain now resumes in parallel past it
    (k_huge_resolve + a fresh set of pointer-jumping rounds, up to HUGE_RESUME_PASSES times): a long
    group at offset 0 followed by 8k vote records, two groups, and four-plus groups (the last ones
    then taken by the serial tail) all equal the prost oracle."""
    from wire_fuzz import random_vote
    from hashgraph_like_consensus.protos import Proposal
    rnd = random.Random(41)
    grp = b"\xfb\x01\x0a\x90\x02" + bytes(272) + b"\xfc\x01"
    votes = [random_vote(rnd) for _ in range(8000)]
    body = encode_proposal(Proposal(name="lg", proposal_id=5, votes=votes, expected_voters_count=30000,
                                    timestamp=3, expiration_timestamp=90))
    msgs = [
        grp + body,
        grp + grp + body + b"\x60\x2d",
        grp * 6 + body,
        encode_proposal(random_proposal(rnd, max_votes=2)),
    ]
    assert all(len(m) > (1 << 20) for m in msgs[:3])
    _check_decode(engine, msgs, _scope(1))
