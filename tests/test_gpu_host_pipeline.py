"""The pipelined host-buffer entry (hlc_validate_proposals cut into proposal chunks that take turns
on 2-4 child contexts, HLC_PIPE_DEPTH; hlc_api.cpp validate_pipelined) equals the one-shot path and the C
oracle bit for bit: per-proposal results, per-vote statuses, scheme reasons and recovered
addresses, on a Byzantine batch; also with empty proposals, votes no proposal covers (gaps between
chunks: status 0xFF), a batch whose proposal ranges are out of order (the one-shot fallback), and
an out-of-arena field in a late chunk (HLC_EINVAL, no device access)."""
import os

import numpy as np
import pytest

import coracle
from adversarial import byzantine
from hashgraph_like_consensus import _ffi
from helpers import oracle_workload

pytestmark = pytest.mark.gpu


def _run(engine, batch, desc, now, chunk, depth=None):
    os.environ["HLC_PIPE_CHUNK_VOTES"] = str(chunk)
    if depth is not None:
        os.environ["HLC_PIPE_DEPTH"] = str(depth)
    try:
        return engine.validate_proposals(batch, desc, now, want_votes=True, want_recovered=True)
    finally:
        os.environ.pop("HLC_PIPE_CHUNK_VOTES", None)
        os.environ.pop("HLC_PIPE_DEPTH", None)


@pytest.fixture(scope="module")
def byz():
    w = oracle_workload(40, 24, 24, True, 0x484C4351, name="pipe")
    b, d, _ = byzantine(w, fraction=1 / 4, seed=0x51)
    return b, d, w.now


@pytest.mark.parametrize("chunk,depth", [(100, 3), (240, 3), (333, 3), (100, 2), (100, 4)])
def test_gpu_pipeline_equals_one_shot_and_oracle(engine, byz, chunk, depth):
    b, d, now = byz
    one = _run(engine, b, d, now, 0)
    pip = _run(engine, b, d, now, chunk, depth)
    for x, y in zip(one, pip):
        assert np.array_equal(x, y)
    cres, cvst, cvrs, crec = coracle.validate_proposals(b, d, now, threads=8)
    assert np.array_equal(pip[0], cres) and np.array_equal(pip[1], cvst)
    assert np.array_equal(pip[2], cvrs) and np.array_equal(pip[3], crec)
    assert len({int(s) for s in pip[0]["status"]}) > 3


def test_gpu_pipeline_gaps_and_empty_proposals(engine, byz):
    b, d, now = byz
    d2 = d.copy()
    d2["vote_count"][3] = 0            # an empty proposal (StillActive)
    d2["vote_count"][10] -= 5          # its last 5 votes are covered by no proposal
    d2["vote_count"][25] = 0
    one = _run(engine, b, d2, now, 0)
    pip = _run(engine, b, d2, now, 100)
    for x, y in zip(one, pip):
        assert np.array_equal(x, y)
    gap = int(d2["vote_begin"][10] + d2["vote_count"][10])
    assert (pip[1][gap:gap + 5] == 0xFF).all()


def test_gpu_pipeline_out_of_order_falls_back(engine, byz):
    b, d, now = byz
    d2 = d[::-1].copy()  # proposals listed in reverse vote order: chunks would interleave
    one = _run(engine, b, d2, now, 0)
    pip = _run(engine, b, d2, now, 100)
    for x, y in zip(one, pip):
        assert np.array_equal(x, y)


def test_gpu_pipeline_rejects_bad_field_in_late_chunk(engine, byz):
    b, d, now = byz
    off = b.field_off.copy()
    off[b.n - 3, 4] = b.arena.size + 10  # signature past the arena, in the last chunk
    bad = b.__class__(b.vote_id, b.proposal_id, b.timestamp, b.vote, b.arena, off, b.field_len)
    with pytest.raises(_ffi.HlcError):
        _run(engine, bad, d, now, 100)
    ok = _run(engine, b, d, now, 100)  # the context is still usable
    assert np.array_equal(ok[1], _run(engine, b, d, now, 0)[1])
