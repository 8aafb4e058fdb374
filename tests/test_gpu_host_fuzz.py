"""Randomised schedules of the host-buffer entries (hlc_api.cpp validate_host / verify_host): for a
Byzantine batch, random proposal subsets in random order, random recovery ranges
(HLC_OPT_SPLIT_VOTES), staging pieces (HLC_OPT_REST_PIECES), first-range prep batches (HLC_OPT_FIRST_BATCH)
and host pool sizes (HLC_OPT_HOST_THREADS), set per context with hlc_ctx_set_option, must give exactly the single-range result -- itself pinned to
the C oracle in test_gpu_host_pipeline.py -- and, for a sample of the settings, the oracle again."""
import os
import random

import numpy as np
import pytest

import coracle
from adversarial import byzantine
from helpers import oracle_workload

pytestmark = pytest.mark.gpu
def _call(engine, batch, desc, now, opts):
    with engine.options(**opts):  # hlc_ctx_set_option: the context's tunables for this call
        return engine.validate_proposals(batch, desc, now, want_votes=True, want_recovered=True)


@pytest.fixture(scope="module")
def big_byz():
    w = oracle_workload(120, 24, 24, True, 0x484C4360, name="fuzz")
    b, d, _ = byzantine(w, fraction=1 / 4, seed=0x60)
    return b, d, w.now


def test_gpu_host_entry_random_schedules(engine, big_byz):
    b, d, now = big_byz
    rnd = random.Random(0x484C)
    for trial in range(16):
        p0 = rnd.randrange(0, d.shape[0] - 1)
        p1 = rnd.randrange(p0 + 1, d.shape[0] + 1)
        sub = d[p0:p1].copy()
        if rnd.random() < 0.5:
            sub = sub[np.array(rnd.sample(range(sub.shape[0]), sub.shape[0]))]
        sizes = [rnd.choice([1, 7, 64, 65, 100, 333, 640, 1000]) for _ in range(rnd.randrange(1, 4))]
        env = {"split_votes": sizes, "rest_pieces": rnd.randrange(1, 9), "first_batch": rnd.randrange(1, 9),
               "host_threads": rnd.randrange(1, 13)}
        ref = _call(engine, b, sub, now, {"split_votes": 0})
        got = _call(engine, b, sub, now, env)
        for x, y in zip(ref, got):
            assert np.array_equal(x, y), (trial, env, p0, p1)
        if trial % 5 == 0:
            cres, cvst, cvrs, crec = coracle.validate_proposals(b, sub, now, threads=8)
            assert np.array_equal(got[0], cres) and np.array_equal(got[1], cvst), (trial, env)
            assert np.array_equal(got[2], cvrs) and np.array_equal(got[3], crec), (trial, env)


def test_gpu_verify_batch_random_schedules(engine):
    """hlc_eth_verify_batch under random ranges / pieces / first-range batch / pool size: every item
    equals the oracle (adversarial items: bad lengths, high s, bad v, no point, wrong key)."""
    from test_gpu_parity import _mutated_items, _oracle_verify
    ids, pays, sigs = _mutated_items(900, 0x61)
    exp_st, exp_addr = _oracle_verify(ids, pays, sigs)
    rnd = random.Random(0x61)
    for trial in range(10):
        n = rnd.randrange(1, len(ids) + 1)
        sizes = [rnd.choice([1, 5, 64, 100, 257]) for _ in range(rnd.randrange(1, 4))]
        env = {"split_votes": sizes, "rest_pieces": rnd.randrange(1, 9), "first_batch": rnd.randrange(1, 9),
               "host_threads": rnd.randrange(1, 13)}
        with engine.options(**env):
            st, addr = engine.eth_verify_batch(ids[:n], pays[:n], sigs[:n])
        assert [int(x) for x in st] == exp_st[:n], (trial, env, n)
        assert [a.tobytes() for a in addr] == exp_addr[:n], (trial, env, n)
