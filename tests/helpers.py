"""Shared test helpers: oracle-backed signers for the synthetic generator, conversions."""
from __future__ import annotations

import numpy as np

import coracle
from hashgraph_like_consensus import synth


def oracle_addr_fn(priv: np.ndarray) -> np.ndarray:
    return coracle.address_batch(priv, threads=8)


def oracle_sign_fn(priv, arena, off, lens, total):
    pre = np.zeros((priv.shape[0], 32), np.uint8)
    for i in range(priv.shape[0]):
        o, l = int(off[i]), int(lens[i])
        pre[i] = np.frombuffer(coracle.eip191_hash(arena[o:o + l].tobytes()), np.uint8)
    return coracle.sign_batch(priv, pre, threads=8)


def oracle_workload(n_props, votes, expected, gossipsub, seed, start=0, name=""):
    return synth.generate(n_props, votes, expected, gossipsub, seed, oracle_addr_fn, oracle_sign_fn,
                          start_proposal=start, name=name)
