"""The checked recovery chains on the GPU.  k_rec_main runs its u2 R and u1 G chains with the
unchecked mixed addition and reroutes a vote through the checked chains (every addition tests
a == +-b) only when a final Z is zero (hlc_recover.hpp rec_u2r29 / rec_comb29).  Crafted inputs that reach
that route cannot be built for the shipped comb (tests/crypto_items.py
comb_collisions_possible), so a context created with HLC_REC_FORCE_EXACT=1 sends EVERY vote
through the checked chains: its outcomes must equal the default context's and the oracle's,
bit for bit (adversarial signature items including crafted Q = infinity, and a Byzantine
config-5-style batch)."""
import os

import numpy as np
import pytest

import coracle
import pyoracle as po
from adversarial import byzantine
from crypto_items import make_items
from helpers import oracle_workload

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def exact_engine():
    from hashgraph_like_consensus.engine import Engine
    eng = Engine(0)
    eng.set_option("rec_force_exact", 1)  # HLC_OPT_REC_FORCE_EXACT: every vote through the checked chains
    yield eng
    eng.close()


def test_gpu_checked_chains_on_adversarial_items(engine, exact_engine):
    items = make_items(3000, 0xE4AC7)
    owners = [po.privkey_to_address(it.priv) for it in items]
    args = (owners, [it.payload for it in items], [it.sig for it in items])
    st_f, addr_f = engine.eth_verify_batch(*args)
    st_x, addr_x = exact_engine.eth_verify_batch(*args)
    assert np.array_equal(np.asarray(st_f), np.asarray(st_x))
    assert np.array_equal(np.asarray(addr_f), np.asarray(addr_x))
    for i, it in enumerate(items):
        code, addr = coracle.ecrecover(it.prehash, it.sig)
        want = (1 + code) if code else (0 if addr == owners[i] else 1)
        assert int(st_x[i]) == want, (i, it.kind)


def test_gpu_checked_chains_validate_many(exact_engine):
    w = oracle_workload(150, 64, 64, True, 0xE4AC8)
    batch, desc, _ = byzantine(w, fraction=1 / 3, seed=0xE4AC8)
    res, vst, vrs, rec = exact_engine.validate_proposals(batch, desc, w.now, want_recovered=True)
    cres, cvst, cvrs, crec = coracle.validate_proposals(batch, desc, w.now)
    assert np.array_equal(vst, cvst) and np.array_equal(vrs, cvrs) and np.array_equal(rec, crec)
    assert np.array_equal(res, cres)
