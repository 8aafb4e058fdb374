"""GPU parity of the streaming vote path (hlc_process_votes through the C ABI, hlc_stream.hip)
against oracle/stream_oracle.py (process_incoming_vote, service.rs:286-305, restated): per-vote
status / transition / inserted / scheme reason and every session's final state, bit for bit,
on micro-batches that mix sessions, replays, Byzantine votes, decided / Failed / expiring
sessions, P2P round limits and storage misses.  Also: a batch split in two consecutive calls
(sessions and owner maps carried over by the caller) ends exactly where one call does.
"""
import numpy as np
import pytest

import pyoracle as po
from stream_cases import device_inputs, run_oracle, sessions_array, streaming_workload

pytestmark = pytest.mark.gpu


def _check(engine, sessions, votes, vs, now):
    ss_ref, out_ref = run_oracle(sessions, votes, vs, now)
    batch, vsess, sarr, owners, osess = device_inputs(sessions, votes, vs)
    st, tr, ins, rs = engine.process_votes(batch, vsess, sarr, owners, osess, now)
    exp = np.array([(o[0], o[1], int(o[2]), o[3]) for o in out_ref], np.int64)
    got = np.stack([st, tr, ins, rs], axis=1).astype(np.int64)
    bad = np.nonzero((exp != got).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} votes differ, first {bad[:5]}: gpu {got[bad[:3]]} ref {exp[bad[:3]]}"
    assert np.array_equal(sarr, sessions_array(ss_ref)), "final session states differ"
    return ss_ref, out_ref


@pytest.mark.parametrize("seed", [0x484C4331, 0x484C4332, 0x484C4333])
def test_gpu_stream_matches_oracle(engine, seed):
    sessions, votes, vs, now = streaming_workload(seed)
    ss_ref, out_ref = _check(engine, sessions, votes, vs, now)
    codes = {o[0] for o in out_ref}
    assert {po.OK, po.DUPLICATE_VOTE, 19} <= codes
    assert any(o[2] for o in out_ref)


def test_gpu_stream_two_calls_equal_one(engine):
    sessions, votes, vs, now = streaming_workload(0x484C4334, n_props=16, votes=10)
    ss_ref, out_ref = run_oracle(sessions, votes, vs, now)
    h = len(votes) // 2
    ss_mid, out_a = run_oracle(sessions, votes[:h], vs[:h], now)
    ss_end, out_b = _check(engine, ss_mid, votes[h:], vs[h:], now)  # caller carries states + owner maps
    assert out_a + out_b == out_ref
    assert np.array_equal(sessions_array(ss_end), sessions_array(ss_ref))


def test_gpu_stream_empty(engine):
    sessions, votes, vs, now = streaming_workload(0x484C4335, n_props=4, votes=4)
    batch, vsess, sarr, owners, osess = device_inputs(sessions, votes[:0], vs[:0])
    before = sarr.copy()
    st, tr, ins, rs = engine.process_votes(batch, vsess, sarr, owners, osess, now)
    assert st.size == 0 and np.array_equal(sarr, before)
