"""GPU parity of the pipelined wire entry (hlc_validate_wire_proposals from host buffers, hlc_api.cpp
validate_wire_host): gossip bytes uploaded in message ranges, each range decoded with a vote-index
offset and its signatures recovered as it lands, one validation over every range.

Forced small ranges (HLC_WIRE_SPLIT_BYTES) and pieces (HLC_WIRE_CHUNK) so that small workloads take
many ranges, messages straddle upload pieces, and decode errors sit in later ranges.  Every case is
compared bit for bit with the unpipelined arm of the same entry (HLC_WIRE_PIPELINE=0: the whole
buffer uploaded, then decoded, then validated -- the path the other wire tests pin to the oracles)
and, where the workload is the oracle's, with the C oracle's from_proposal outcomes
(consensus.proto:5-29 decoded as prost does, then service.rs:263-279 / session.rs:198-221).
"""
import contextlib
import os
import random

import numpy as np
import pytest

import coracle
import wire_oracle as wo
from adversarial import byzantine
from hashgraph_like_consensus import _ffi, synth
from hashgraph_like_consensus.protos import Proposal, encode_proposal
from helpers import oracle_workload
from wire_fuzz import mutate, random_proposal

pytestmark = pytest.mark.gpu
THREADS = max(1, min(16, os.cpu_count() or 1))


_OPT = {"HLC_WIRE_SPLIT_BYTES": "wire_split_bytes", "HLC_WIRE_CHUNK": "wire_chunk",
        "HLC_WIRE_PIPELINE": "wire_pipeline", "HLC_HOST_TRACE": "host_trace"}


def _env(engine, **kw):
    """The context's wire tunables for a block (hlc_ctx_set_option), named by their environment defaults."""
    return engine.options(**{_OPT[k]: (v if k == "HLC_WIRE_SPLIT_BYTES" else int(v)) for k, v in kw.items()})


def _scope(n, gossipsub=True):
    sc = np.zeros(n, _ffi.SCOPE_CONFIG_DTYPE)
    sc["consensus_threshold"] = 2.0 / 3.0
    sc["max_rounds"] = 2 if gossipsub else 0
    sc["use_gossipsub_rounds"] = 1 if gossipsub else 0
    return sc


def _pack(msgs):
    lens = np.array([len(m) for m in msgs], np.uint32)
    off = np.zeros(len(msgs), np.uint64)
    if msgs:
        off[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
    return np.frombuffer(b"".join(msgs) or b"\0", np.uint8)[:int(lens.sum())].copy(), off, lens


def _both(engine, wire, off, lens, scope, now, split="4096,8192", chunk=3000, min_ranges=2):
    """(pipelined, unpipelined) outcomes of one call; asserts they are equal bit for bit, and that the
    pipelined call took at least `min_ranges` message ranges (its HLC_HOST_TRACE facts).  Returns
    (results, wire info, decoded votes, the pipelined call's trace facts)."""
    with _env(engine, HLC_WIRE_SPLIT_BYTES=split, HLC_WIRE_CHUNK=chunk, HLC_WIRE_PIPELINE=1, HLC_HOST_TRACE=2):
        pr, pw, pn = engine.validate_wire_proposals(wire, off, lens, scope, now)
        facts = engine.last_host_trace()["facts"]
    with _env(engine, HLC_WIRE_PIPELINE=0):
        ur, uw, un = engine.validate_wire_proposals(wire, off, lens, scope, now)
    assert pn == un, f"decoded votes {pn} != {un}"
    bad = np.nonzero(pr != ur)[0]
    assert bad.size == 0, f"{bad.size} results differ from the unpipelined entry, first {bad[:5]}"
    assert np.array_equal(pw.view(np.uint8), uw.view(np.uint8)), "wire info differs from the unpipelined entry"
    assert facts["ranges"] >= min_ranges, facts
    return pr, pw, pn, facts


def _with_extra(w_batch, desc, extra, every=5):
    """The workload's messages with undecodable ones interleaved (one after every `every` messages),
    so that decode errors fall into the middle and the later ranges."""
    wire, off, lens, _ = synth.to_wire(w_batch, desc)
    msgs = [wire[int(o):int(o) + int(n)].tobytes() for o, n in zip(off, lens)]
    out, where = [], []
    ex = list(extra)
    for i, m in enumerate(msgs):
        out.append(m)
        where.append(("ok", i))
        if (i + 1) % every == 0 and ex:
            out.append(ex.pop(0))
            where.append(("extra", None))
    for m in ex:
        out.append(m)
        where.append(("extra", None))
    return out, where


def test_gpu_wire_pipeline_ranges_and_late_decode_errors(engine):
    """48 proposals x 16 votes in ranges of 4 KiB, 8 KiB, doubling (pieces of 3,000 B, so messages
    straddle pieces), with 20 undecodable messages interleaved -- decode errors in later ranges --
    equal to the unpipelined entry and to the oracle (decoded messages) and the prost oracle (the
    undecodable ones: status 17, the prost error code, the failing record)."""
    w = oracle_workload(48, 16, 16, True, 0x484C4351, name="wire-pipe")
    rnd = random.Random(51)
    extra = [mutate(rnd, encode_proposal(random_proposal(rnd, max_votes=3))) for _ in range(20)]
    msgs, where = _with_extra(w.batch, w.desc, extra)
    wire, off, lens = _pack(msgs)
    assert wire.size > 8 * 4096  # several ranges
    res, winfo, nv, _ = _both(engine, wire, off, lens, _scope(1), w.now, min_ranges=4)
    cres, _, _, _ = coracle.validate_proposals(w.batch, w.desc, w.now, threads=THREADS)
    for m, (kind, i) in enumerate(where):
        if kind == "ok":
            assert res[m] == cres[i], f"message {m} (proposal {i}) differs from the oracle"
            assert int(winfo[m]["decode_status"]) == 0
        else:
            code, _, badv = wo.decode_proposal_ex(msgs[m])
            if code != wo.OK:
                assert (int(res[m]["status"]), int(res[m]["scheme_reason"]), int(res[m]["bad_index"])) == (
                    17, code, badv), f"message {m}: decode error outcome"
    assert (res["status"][[m for m, (k, _) in enumerate(where) if k == "ok"]] == 0).all()


def test_gpu_wire_pipeline_byzantine_many_ranges(engine):
    """A Byzantine batch (1/3 of the votes mutated) over many small ranges == the oracle."""
    w = oracle_workload(64, 16, 16, True, 0x484C4352, name="wire-pipe-byz")
    batch, desc, kinds = byzantine(w, fraction=1 / 3, seed=11)
    wire, off, lens, scope = synth.to_wire(batch, desc)
    res, _, _, _ = _both(engine, wire, off, lens, scope, w.now, split="2048", chunk=1024, min_ranges=4)
    cres, _, _, _ = coracle.validate_proposals(batch, desc, w.now, threads=THREADS)
    assert np.array_equal(res, cres)
    assert (res["status"] != 0).sum() > 0


def test_gpu_wire_pipeline_out_of_order_and_overlap(engine):
    """Messages laid out in reverse order in the buffer (the first range's byte prefix is then the
    whole buffer), a message referenced twice, empty messages with offsets past the buffer, and a
    per-message scope array."""
    w = oracle_workload(24, 8, 8, True, 0x484C4353, name="wire-pipe-order")
    wire, off, lens, scope = synth.to_wire(w.batch, w.desc)
    P = off.size
    perm = np.arange(P)[::-1]
    msgs = [wire[int(off[i]):int(off[i]) + int(lens[i])].tobytes() for i in perm]
    rw, roff, rlen = _pack(msgs)
    # message k of the call = proposal k, whose bytes now sit at the mirrored place
    off2 = np.array([roff[P - 1 - k] for k in range(P)], np.uint64)
    len2 = lens.copy()
    off2 = np.concatenate([off2, off2[:1], np.array([10 ** 12, 7], np.uint64)])
    len2 = np.concatenate([len2, len2[:1], np.array([0, 0], np.uint32)])
    sc = _scope(P + 3)
    sc["max_rounds"][P + 1:] = 5
    res, _, nv, _ = _both(engine, rw, off2, len2, sc, w.now, split="3000,3000", chunk=2048, min_ranges=1)
    cres, _, _, _ = coracle.validate_proposals(w.batch, w.desc, w.now, threads=THREADS)
    assert np.array_equal(res[:P], cres)
    assert res[P] == res[0]  # the repeated message validates on its own, as the first
    assert nv == int(w.batch.n) + int(w.desc["vote_count"][0])


def test_gpu_wire_pipeline_big_messages_in_later_ranges(engine):
    """Messages with more vote records than the walker keeps per message (128), placed in later
    ranges (the range's second walk writes them at its vote base), one corrupted."""
    from wire_fuzz import random_vote
    rnd = random.Random(53)
    msgs = [encode_proposal(random_proposal(rnd, max_votes=3)) for _ in range(30)]
    for k in range(3):
        msgs.append(encode_proposal(Proposal(name="big", proposal_id=500 + k, expected_voters_count=900,
                                             votes=[random_vote(rnd) for _ in range(150 + 40 * k)],
                                             timestamp=5, expiration_timestamp=9)))
        msgs += [encode_proposal(random_proposal(rnd, max_votes=3)) for _ in range(10)]
    big = bytearray(msgs[31 + 11])
    big[len(big) // 2] ^= 0x80
    msgs[31 + 11] = bytes(big)
    wire, off, lens = _pack(msgs)
    _both(engine, wire, off, lens, _scope(1), 1_760_001_800, split="6000", chunk=4096)


def test_gpu_wire_pipeline_density_overflow_falls_back():
    """The first range holds no votes (a large payload) and the later ones thousands of 2-byte vote
    records: more votes than the first range's density promised, so the call drains and re-runs
    unpipelined -- same outcomes; the next call of that size fits its capacity."""
    from hashgraph_like_consensus.engine import Engine
    eng = Engine(0)  # a fresh context: no vote-count hint from earlier calls
    try:
        head = encode_proposal(Proposal(name="sparse", payload=bytes(20_000), proposal_id=1))
        msgs = [head] + [encode_proposal(Proposal(proposal_id=2 + k, expected_voters_count=9)) + b"\x72\x00" * 3000
                         for k in range(16)]
        wire, off, lens = _pack(msgs)
        r1 = _both(eng, wire, off, lens, _scope(1), 1_760_001_800, split="20000,8000", chunk=8192)
        assert "overflow_capacity" in r1[3], r1[3]  # drained and re-run unpipelined
        r2 = _both(eng, wire, off, lens, _scope(1), 1_760_001_800, split="20000,8000", chunk=8192)
        assert "overflow_capacity" not in r2[3] and r2[3]["capacity"] >= r2[2], r2[3]
        assert np.array_equal(r1[0], r2[0]) and r1[2] == r2[2] and r1[2] >= 16 * 3000
    finally:
        eng.close()


def test_gpu_wire_pipeline_pinned_wire(engine):
    """The gossip bytes in page-locked memory (hlc_host_alloc): the ranges are DMA'd straight from
    the caller's buffer -- same outcomes."""
    w = oracle_workload(16, 8, 8, True, 0x484C4354, name="wire-pipe-pinned")
    wire, off, lens, scope = synth.to_wire(w.batch, w.desc)
    arena = _ffi.PinnedArena(wire.size + 64)
    pw = arena.take(wire.shape, np.uint8)
    pw[:] = wire
    res, _, _, facts = _both(engine, pw, off, lens, scope, w.now, split="2000", chunk=1500)
    assert facts["wire_pinned"] == 1
    cres, _, _, _ = coracle.validate_proposals(w.batch, w.desc, w.now, threads=THREADS)
    assert np.array_equal(res, cres)
    arena.close()


def test_gpu_wire_pipeline_bad_extent_outputs_untouched(engine):
    """A message extent outside the wire buffer: HLC_EINVAL before anything runs, outputs untouched."""
    import ctypes
    from ctypes import c_uint8, c_uint32, c_uint64, c_void_p
    w = oracle_workload(4, 8, 8, True, 0x484C4355, name="wire-pipe-einval")
    wire, off, lens, scope = synth.to_wire(w.batch, w.desc)
    off = off.copy()
    off[3] = wire.size  # the last message now runs past the end
    resb = np.full(4 * 16, 0xAB, np.uint8)
    wi = np.full(4 * 48, 0xCD, np.uint8)
    nv = c_uint64(77)
    with _env(engine, HLC_WIRE_SPLIT_BYTES="512", HLC_WIRE_CHUNK=512):
        rc = engine.lib.hlc_validate_wire_proposals(
            engine.ctx, _ffi.ptr(wire, c_uint8), wire.size, _ffi.ptr(off, c_uint64), _ffi.ptr(lens, c_uint32), 4,
            c_void_p(scope.ctypes.data), scope.shape[0], w.now, c_void_p(resb.ctypes.data), c_void_p(wi.ctypes.data),
            ctypes.byref(nv))
    assert rc == -1  # HLC_EINVAL
    assert (resb == 0xAB).all() and (wi == 0xCD).all() and nv.value == 77
    # the context is still good
    _both(engine, *synth.to_wire(w.batch, w.desc), w.now, split="512", chunk=512)


def test_gpu_wire_pipeline_fuzzed_schedules(engine):
    """Random range schedules (1-3 listed sizes of 1-48 KiB, then doubling) and upload pieces (512 B -
    16 KiB) over a mix of valid signed proposals, fuzzed proposals (every prost error class, some with
    more than 128 vote records) and empty messages, in buffer order or shuffled: the pipelined entry
    equals the unpipelined one bit for bit every time."""
    from wire_fuzz import random_vote
    rnd = random.Random(61)
    w = oracle_workload(40, 8, 8, True, 0x484C4356, name="wire-pipe-fuzz")
    wire0, off0, lens0, _ = synth.to_wire(w.batch, w.desc)
    good = [wire0[int(o):int(o) + int(n)].tobytes() for o, n in zip(off0, lens0)]
    for trial in range(6):
        msgs = []
        for t in range(120):
            k = rnd.randrange(10)
            if k < 4:
                msgs.append(rnd.choice(good))
            elif k < 8:
                msgs.append(mutate(rnd, encode_proposal(random_proposal(rnd, max_votes=4))))
            elif k == 8:
                msgs.append(encode_proposal(Proposal(name="b", proposal_id=9000 + t, expected_voters_count=400,
                                                     votes=[random_vote(rnd) for _ in range(130)])))
            else:
                msgs.append(b"")
        wire, off, lens = _pack(msgs)
        if trial % 2:  # messages laid out in another order than the call lists them
            perm = list(range(len(msgs)))
            rnd.shuffle(perm)
            wire, poff, plens = _pack([msgs[i] for i in perm])
            inv = {p: j for j, p in enumerate(perm)}
            off = np.array([poff[inv[i]] for i in range(len(msgs))], np.uint64)
            lens = np.array([plens[inv[i]] for i in range(len(msgs))], np.uint32)
        split = ",".join(str(rnd.randrange(1024, 48 * 1024)) for _ in range(rnd.randrange(1, 4)))
        _both(engine, wire, off, lens, _scope(1), w.now, split=split, chunk=rnd.randrange(512, 16384),
              min_ranges=1)
