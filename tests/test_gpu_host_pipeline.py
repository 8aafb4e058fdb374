"""The host-buffer entry hlc_validate_proposals (hlc_api.cpp validate_host: the signatures staged
and uploaded first as a dense array, range by range, each range's k_rec_prep + k_rec_main behind its
upload on two streams in turn, the other inputs in pieces behind them) equals the single-range
schedule and the C oracle bit for bit:
per-proposal results, per-vote statuses, scheme reasons and recovered addresses, on a Byzantine
batch; also with empty proposals, votes no proposal covers (status 0xFF), proposals listed out of
vote order, and an out-of-arena field -- a signature in the second range or another field in a late
piece -- which returns HLC_EINVAL with the caller's outputs untouched (the device work already
enqueued is drained and discarded).  Schedule knobs: HLC_SPLIT_VOTES (sizes of the recovery ranges
before the last, "0" = one range), HLC_REST_PIECES, HLC_FIRST_BATCH."""
import ctypes
import os

import numpy as np
import pytest

import coracle
from adversarial import byzantine
from hashgraph_like_consensus import _ffi
from hashgraph_like_consensus.batch import proposals_ptr, results_ptr
from helpers import oracle_workload

pytestmark = pytest.mark.gpu
HLC_EINVAL = -1  # include/hlc.h


def _run(engine, batch, desc, now, split, pieces=None):
    opts = {"split_votes": str(split)}
    if pieces is not None:
        opts["rest_pieces"] = pieces
    with engine.options(**opts):
        return engine.validate_proposals(batch, desc, now, want_votes=True, want_recovered=True)


@pytest.fixture(scope="module")
def byz():
    w = oracle_workload(40, 24, 24, True, 0x484C4351, name="pipe")
    b, d, _ = byzantine(w, fraction=1 / 4, seed=0x51)
    return b, d, w.now


@pytest.mark.parametrize("split,pieces", [("100", 3), ("240", 1), ("333", 7), ("1", 2), ("1,1,1,1", 64), ("64,128", 3),
                                          ("100,150,90", 5), ("32,32,32,32,32,32,32", 1)])
def test_gpu_host_entry_equals_single_range_and_oracle(engine, byz, split, pieces):
    b, d, now = byz
    one = _run(engine, b, d, now, 0, 1)
    got = _run(engine, b, d, now, split, pieces)
    for x, y in zip(one, got):
        assert np.array_equal(x, y)
    cres, cvst, cvrs, crec = coracle.validate_proposals(b, d, now, threads=8)
    assert np.array_equal(got[0], cres) and np.array_equal(got[1], cvst)
    assert np.array_equal(got[2], cvrs) and np.array_equal(got[3], crec)
    assert len({int(s) for s in got[0]["status"]}) > 3


@pytest.mark.parametrize("first_batch", ["1", "2", "3", "8"])
def test_gpu_host_entry_first_range_prep_batch(engine, byz, first_batch):
    """The first range's k_rec_prep with 1, 2, 3 or 8 votes per lane (HLC_FIRST_BATCH: the lane count
    and the prefix-product layout follow it) equals the oracle bit for bit."""
    b, d, now = byz
    with engine.options(first_batch=int(first_batch)):
        got = _run(engine, b, d, now, "100,150")
        one = _run(engine, b, d, now, "0")
    for x, y in zip(one, got):
        assert np.array_equal(x, y)
    cres, cvst, cvrs, crec = coracle.validate_proposals(b, d, now, threads=8)
    assert np.array_equal(got[0], cres) and np.array_equal(got[1], cvst)
    assert np.array_equal(got[2], cvrs) and np.array_equal(got[3], crec)


def test_gpu_host_entry_gaps_and_empty_proposals(engine, byz):
    b, d, now = byz
    d2 = d.copy()
    d2["vote_count"][3] = 0            # an empty proposal (StillActive)
    d2["vote_count"][10] -= 5          # its last 5 votes are covered by no proposal
    d2["vote_count"][25] = 0
    one = _run(engine, b, d2, now, 0)
    got = _run(engine, b, d2, now, 100)
    for x, y in zip(one, got):
        assert np.array_equal(x, y)
    cres, cvst, _, _ = coracle.validate_proposals(b, d2, now, threads=8)
    assert np.array_equal(got[0], cres) and np.array_equal(got[1], cvst)
    gap = int(d2["vote_begin"][10] + d2["vote_count"][10])
    assert (got[1][gap:gap + 5] == 0xFF).all()


def test_gpu_host_entry_out_of_order_proposals(engine, byz):
    b, d, now = byz
    d2 = d[::-1].copy()  # proposals listed in reverse vote order
    one = _run(engine, b, d2, now, 0)
    got = _run(engine, b, d2, now, 100)
    for x, y in zip(one, got):
        assert np.array_equal(x, y)
    cres, _, _, _ = coracle.validate_proposals(b, d2, now, threads=8)
    assert np.array_equal(got[0], cres)


def _raw_call(engine, batch, desc, now, split):
    """hlc_validate_proposals through ctypes with outputs pre-filled with 0xAB: -> (rc, outputs)."""
    n = batch.n
    res = np.full(desc.shape[0], 0xAB, np.uint8).repeat(16).view(_ffi.RESULT_DTYPE)
    st = np.full(n, 0xAB, np.uint8)
    rs = np.full(n, 0xAB, np.uint8)
    rec = np.full((n, 20), 0xAB, np.uint8)
    view = batch.view()
    desc = np.ascontiguousarray(desc)
    with engine.options(split_votes=str(split)):
        rc = engine.lib.hlc_validate_proposals(engine.ctx, ctypes.byref(view), proposals_ptr(desc), desc.shape[0], now,
                                               results_ptr(res), _ffi.ptr(st, ctypes.c_uint8),
                                               _ffi.ptr(rs, ctypes.c_uint8), _ffi.ptr(rec, ctypes.c_uint8))
    return rc, (res.view(np.uint8), st, rs, rec)


@pytest.mark.parametrize("field,where,far", [(4, "second range", False), (2, "late piece", False),
                                             (0, "late piece", False), (4, "second range", True),
                                             (1, "late piece", True), (3, "late piece", True)])
def test_gpu_host_entry_rejects_bad_field_outputs_untouched(engine, byz, field, where, far):
    """far: an offset of 2^40, which a kernel reading the field would fault on -- the check must come
    before any kernel that reads the field is enqueued."""
    b, d, now = byz
    off = b.field_off.copy()
    # a vote in the second recovery range and in the last staging piece whose field is non-empty
    i = max(j for j in range(b.n - 20, b.n) if int(b.field_len[j, field]) > 0)
    off[i, field] = (1 << 40) if far else b.arena.size + 10
    bad = b.__class__(b.vote_id, b.proposal_id, b.timestamp, b.vote, b.arena, off, b.field_len)
    rc, outs = _raw_call(engine, bad, d, now, 100)
    assert rc == HLC_EINVAL, where
    for o in outs:
        assert (o == 0xAB).all(), "outputs were written on error"
    ok = _run(engine, b, d, now, 100)  # the context is still usable
    assert np.array_equal(ok[1], _run(engine, b, d, now, 0)[1])


def test_gpu_host_entry_pinned_inputs(engine, byz):
    """Inputs the caller built in page-locked memory (hlc_host_alloc) are DMA'd without the staging
    copy: all arrays pinned, or only some (the library checks each one), equal the pageable call and
    the oracle bit for bit."""
    b, d, now = byz
    ref = _run(engine, b, d, now, "100")
    pb = b.pinned()
    got = _run(engine, pb, d, now, "100")
    for x, y in zip(ref, got):
        assert np.array_equal(x, y)
    mixed = b.__class__(b.vote_id, pb.proposal_id, b.timestamp, pb.vote, pb.arena, b.field_off, pb.field_len)
    got2 = _run(engine, mixed, d, now, "64,128")
    for x, y in zip(ref, got2):
        assert np.array_equal(x, y)
    cres, cvst, cvrs, crec = coracle.validate_proposals(b, d, now, threads=8)
    assert np.array_equal(got[0], cres) and np.array_equal(got[1], cvst)
    assert np.array_equal(got[2], cvrs) and np.array_equal(got[3], crec)


def test_gpu_host_entry_arena_layouts(engine, byz):
    """Arena layouts the range spans must handle: fields of late votes placed first in the arena
    (the first range's span covers almost all of it), votes sharing the same bytes (overlapping
    spans across ranges), and unused garbage around the fields -- all equal the packed layout."""
    b, d, now = byz
    ref = _run(engine, b, d, now, "0")
    n = b.n
    # reversed: vote i's fields move to the mirrored position of the arena
    order = np.arange(n)[::-1]
    chunks, off, pos = [], np.zeros_like(b.field_off), 0
    junk = np.frombuffer(bytes(range(256)) * 4, np.uint8)
    for i in order:
        for f in range(5):
            ln = int(b.field_len[i, f])
            src = b.arena[int(b.field_off[i, f]):int(b.field_off[i, f]) + ln]
            chunks.append(src)
            off[i, f] = pos
            pos += ln
        chunks.append(junk[: (i * 7) % 97])  # garbage between votes
        pos += (i * 7) % 97
    arena = np.concatenate(chunks).astype(np.uint8) if chunks else np.zeros(0, np.uint8)
    rev = b.__class__(b.vote_id, b.proposal_id, b.timestamp, b.vote, arena, off, b.field_len)
    for split in ("100", "64,128"):
        got = _run(engine, rev, d, now, split)
        for x, y in zip(ref, got):
            assert np.array_equal(x, y), split
    # shared bytes: every vote's owner field points at the first vote's owner bytes (an arena region
    # read by every range); only the owners change, so compare with the oracle
    off2 = b.field_off.copy()
    off2[:, 0] = b.field_off[0, 0]
    ln2 = b.field_len.copy()
    ln2[:, 0] = b.field_len[0, 0]
    shared = b.__class__(b.vote_id, b.proposal_id, b.timestamp, b.vote, b.arena, off2, ln2)
    got = _run(engine, shared, d, now, "100")
    one = _run(engine, shared, d, now, "0")
    for x, y in zip(one, got):
        assert np.array_equal(x, y)
    cres, cvst, _, _ = coracle.validate_proposals(shared, d, now, threads=8)
    assert np.array_equal(got[0], cres) and np.array_equal(got[1], cvst)


def test_gpu_host_entry_no_votes(engine):
    """Proposals with no votes at all (an empty batch, no arena): every proposal StillActive, as
    initialize_with_votes on an empty list (session.rs:266-268) -- through the host entry."""
    from hashgraph_like_consensus import _ffi as ffi
    from hashgraph_like_consensus.batch import VoteBatch
    d = np.zeros(3, ffi.PROPOSAL_DTYPE)
    d["proposal_id"] = [1, 2, 3]
    d["timestamp"] = 1_760_000_000
    d["expiration_timestamp"] = 1_760_003_600
    d["expected_voters_count"] = 3
    d["max_rounds"] = 2
    d["consensus_threshold"] = 2 / 3
    d["use_gossipsub_rounds"] = 1
    e = np.zeros(0, np.uint32)
    b = VoteBatch(e, e.copy(), np.zeros(0, np.uint64), np.zeros(0, np.uint8), np.zeros(0, np.uint8),
                  np.zeros((0, 5), np.uint64), np.zeros((0, 5), np.uint32))
    res, _, _, _ = engine.validate_proposals(b, d, 1_760_001_800, want_votes=True)
    cres, _, _, _ = coracle.validate_proposals(b, d, 1_760_001_800, threads=1)
    assert np.array_equal(res, cres)
    assert (res["status"] == 0).all() and (res["transition"] == 0).all()


def _hip_register():
    hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    return hip


def test_gpu_host_entry_split_registration_is_staged(engine, byz):
    """VERDICT r04 item 5 / ADVICE r04: an input array whose first and last bytes are page-locked but
    in two different registrations (two adjacent hipHostRegister blocks, or a first and a last page with
    pageable memory between) is staged, not DMA'd straight from the caller as one block; one
    registration covering the whole array is DMA'd directly.  Outcomes equal the oracle every time
    (the HLC_HOST_TRACE pinned_mask fact shows which arrays went direct: bit 4 = field_off)."""
    b, d, now = byz
    hip = _hip_register()
    page = 4096
    fo = np.ascontiguousarray(b.field_off)
    nb = fo.nbytes
    raw = np.zeros(nb + 3 * page, np.uint8)
    start = (-raw.ctypes.data) % page
    buf = raw[start:start + nb + page]
    view = buf[:nb].view(np.uint64).reshape(fo.shape)
    view[...] = fo
    assert nb > 3 * page
    base = buf.ctypes.data
    mid = (nb // 2) // page * page
    cb = type(b)(b.vote_id, b.proposal_id, b.timestamp, b.vote, b.arena, view, b.field_len)
    cres, cvst, cvrs, crec = coracle.validate_proposals(b, d, now, threads=8)

    def run():
        with engine.options(host_trace=2):
            got = engine.validate_proposals(cb, d, now, want_votes=True, want_recovered=True)
            mask = int(engine.last_host_trace()["facts"]["pinned_mask"])
        assert np.array_equal(got[0], cres) and np.array_equal(got[1], cvst)
        assert np.array_equal(got[2], cvrs) and np.array_equal(got[3], crec)
        return (mask >> 4) & 1

    assert run() == 0  # pageable
    layouts = [[(0, mid), (mid, nb + page - mid)],               # two adjacent registrations
               [(0, page), (nb - nb % page - page, 2 * page)],   # first and last pages, pageable between
               [(0, nb + page)]]                                 # one registration: direct DMA
    for k, regs in enumerate(layouts):
        for o, ln in regs:
            assert hip.hipHostRegister(ctypes.c_void_p(base + o), ln, 0) == 0, (k, o, ln)
        try:
            assert run() == (1 if k == 2 else 0), f"layout {k}"
        finally:
            for o, _ in regs:
                assert hip.hipHostUnregister(ctypes.c_void_p(base + o)) == 0


def test_gpu_pinned_arena_freed_without_gc(engine):
    """the page-locked block of a PinnedArena is released by reference counting once the arena
    and its arrays are gone -- no reference cycle waiting for a garbage-collection pass."""
    import gc
    import weakref
    gc.disable()
    try:
        arena = _ffi.PinnedArena(1 << 20)
        a = arena.take((1000,), np.uint32)
        a[:] = 7
        block = weakref.ref(arena._block)
        del arena
        assert block() is not None and int(a.sum()) == 7000  # the array keeps the block alive
        del a
        assert block() is None  # freed (hlc_host_free) at once
    finally:
        gc.enable()
