"""The config-5 mutation pass signs in one deferred, multithreaded batch (adversarial._Deferred);
its output must be byte-identical to signing at every mutation (mutate without a shared
_Deferred flushes per call).  CPU only, test infrastructure."""
import random

import numpy as np

from adversarial import KINDS, batch_to_votes, byzantine, mutate
from hashgraph_like_consensus.batch import pack_votes
from helpers import oracle_workload


def _immediate(workload, fraction, seed):
    rnd = random.Random(seed)
    votes = batch_to_votes(workload.batch)
    privs = [int.from_bytes(bytes(k), "big") for k in workload.priv]
    k = 0
    for p in range(workload.desc.shape[0]):
        b, c = int(workload.desc[p]["vote_begin"]), int(workload.desc[p]["vote_count"])
        for j in range(c):
            if rnd.random() < fraction:
                mutate(votes, privs, b + j, j, KINDS[k % len(KINDS)], rnd, b, b + c)
                k += 1
    return pack_votes(votes)


def test_deferred_signing_is_byte_identical():
    w = oracle_workload(12, 16, 16, True, 0x484C4399)
    fast, _, kinds = byzantine(w, fraction=0.4, seed=17)
    slow = _immediate(w, 0.4, 17)
    assert set(k for k in kinds if k) == set(KINDS)
    for f in ("vote_id", "proposal_id", "timestamp", "vote", "arena", "field_off", "field_len"):
        assert np.array_equal(getattr(fast, f), getattr(slow, f)), f
