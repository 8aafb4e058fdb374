"""SURVEY.md §8d config 5 (1/3 Byzantine votes) on the device -- the host side.

`hlc_synth_byzantine_device` (hlc_synth.hip k_byz_mutate / k_byz_sign) turns a batch made by
`hlc_synth_votes_device` into the Byzantine mix in place, re-hashing and re-signing on the GPU.
Every mutation kind is BUILT to have one outcome, so the expected per-vote `validate_vote` status
(utils.rs:127-171, with the proposal-id match of utils.rs:113-115) and the expected per-proposal
`from_proposal` first error (session.rs:198-298; SURVEY.md Appendix B precedence) follow from the
mutation plan alone -- no oracle, so bench.py can assert them before it times the mix.  The plan is
recomputed here from the seed (`plan`) and must equal the kinds the device reports.

Kinds (include/hlc.h HLC_BYZ_*; the device kernel's comment gives the construction of each).
A re-hashed vote keeps its successor's received_hash stale (only the Byzantine voter re-signs), so
the successor's received link breaks as well: that is why a chain kind surfaces at its own index.
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np

from .synth import T0, mix

NONE, WRONG_KEY, FLIP_S, BAD_V, HIGH_S, NO_POINT, INFINITY, TAMPER_HASH, SIG_LEN = range(9)
EMPTY_OWNER, EMPTY_HASH, EMPTY_SIG, WRONG_PID, TS_OLD = range(9, 14)
BAD_RECEIVED, TS_REGRESS, PARENT_OTHER, DUPLICATE = range(14, 18)
NAMES = ["none", "wrong_key", "flip_s", "bad_v", "high_s", "no_point", "infinity", "tamper_hash", "sig_len",
         "empty_owner", "empty_hash", "empty_sig", "wrong_pid", "ts_old", "bad_received", "ts_regress",
         "parent_other", "duplicate"]

# HLC_* status codes (include/hlc.h)
OK, PID_MISMATCH, EMPTY_OWNER_ST, EMPTY_HASH_ST, EMPTY_SIG_ST, INVALID_HASH = 0, 2, 3, 4, 5, 6
SCHEME, INVALID_SIG, TS_OLDER, RECEIVED_MISMATCH, PARENT_MISMATCH, DUPLICATE_VOTE = 7, 8, 9, 11, 12, 13
# per-vote (status, HLC_SCHEME_* reason) each kind is built to have
PER_VOTE: Dict[int, Tuple[int, int]] = {
    NONE: (OK, 0), WRONG_KEY: (INVALID_SIG, 0), FLIP_S: (INVALID_SIG, 0), BAD_V: (SCHEME, 3),
    HIGH_S: (OK, 0), NO_POINT: (SCHEME, 5), INFINITY: (SCHEME, 6), TAMPER_HASH: (INVALID_HASH, 0),
    SIG_LEN: (SCHEME, 1), EMPTY_OWNER: (EMPTY_OWNER_ST, 0), EMPTY_HASH: (EMPTY_HASH_ST, 0),
    EMPTY_SIG: (EMPTY_SIG_ST, 0), WRONG_PID: (PID_MISMATCH, 0), TS_OLD: (TS_OLDER, 0),
    BAD_RECEIVED: (OK, 0), TS_REGRESS: (OK, 0), PARENT_OTHER: (OK, 0), DUPLICATE: (OK, 0),
}
REHASHED = (TS_OLD, BAD_RECEIVED, TS_REGRESS, PARENT_OTHER, DUPLICATE)
_CHAIN_MODE = np.array([HIGH_S, BAD_RECEIVED, TS_REGRESS, PARENT_OTHER, DUPLICATE], np.uint8)


def plan(seed: int, start_proposal: int, n_proposals: int, votes_per_proposal: int) -> np.ndarray:
    """The per-vote kinds k_byz_mutate applies (u8[n]), recomputed on the host."""
    P, V = int(n_proposals), int(votes_per_proposal)
    n = P * V
    j = np.tile(np.arange(V, dtype=np.uint64), P)
    p = np.repeat(np.arange(P, dtype=np.uint64), V)
    gidx = (np.uint64(start_proposal) + p) * np.uint64(V) + j
    mode = (mix(seed, 9, np.uint64(start_proposal) + np.arange(P, dtype=np.uint64)) & np.uint64(7)).astype(np.int64)
    mode_v = np.repeat(mode, V)
    mutated = (mix(seed, 7, gidx) % np.uint64(3)) == 0
    h = mix(seed, 8, gidx)
    k_any = (1 + h % np.uint64(17)).astype(np.int64)
    first = j == 0
    k_any = np.where(first & (k_any >= BAD_RECEIVED), (1 + h % np.uint64(13)).astype(np.int64), k_any)
    k_chain = _CHAIN_MODE[(h % np.uint64(5)).astype(np.int64)].astype(np.int64)
    k_chain = np.where(first, HIGH_S, k_chain)
    k = np.where(mode_v <= 3, k_any, np.where(mode_v <= 5, k_chain, HIGH_S))
    k = np.where(mutated, k, NONE)
    last = (j == np.uint64(V - 1)) & (j > 0)
    k = np.where((mode_v == 6) & last, DUPLICATE, k)
    return k.astype(np.uint8).reshape(n)


def expectations(kinds: np.ndarray, votes_per_proposal: int, choice: np.ndarray):
    """-> (vote_status u8[n], vote_reason u8[n] (scheme reason where status == SIGNATURE_SCHEME),
    proposal status u8[P], bad_index u32[P] (0xFFFFFFFF for OK), yes u32[P], total u32[P]) that
    the mutation plan `kinds` (one batch of proposals x V votes, synth.py timestamps) is built to
    produce.  Precedence as from_proposal: the first per-vote failure, then
    the chain (received link before parent at one index), then the first duplicate owner; the
    Gossipsub round limit (n = V, max_rounds 2) never binds."""
    V = int(votes_per_proposal)
    n = kinds.shape[0]
    P = n // V
    lut_s = np.array([PER_VOTE[k][0] for k in range(18)], np.uint8)
    lut_r = np.array([PER_VOTE[k][1] for k in range(18)], np.uint8)
    vst = lut_s[kinds]
    vrs = np.where(vst == SCHEME, lut_r[kinds], 0).astype(np.uint8)
    pst = np.zeros(P, np.uint8)
    bad = np.full(P, 0xFFFFFFFF, np.uint32)
    yes = np.zeros(P, np.uint32)
    total = np.zeros(P, np.uint32)
    jj = np.arange(V)
    ts_orig = T0 + 1 + jj // 1024
    rehashed = np.isin(np.arange(18), REHASHED)
    for p in range(P):
        k = kinds[p * V:(p + 1) * V]
        f = np.nonzero(vst[p * V:(p + 1) * V])[0]
        if f.size:
            pst[p], bad[p] = vst[p * V + f[0]], f[0]
            continue
        ts = np.where(k == TS_REGRESS, T0 + (jj - 1) // 1024, ts_orig)
        done = False
        for j in range(1, V):
            recv_ok = k[j] != BAD_RECEIVED and not rehashed[k[j - 1]] and ts[j - 1] <= ts[j]
            if not recv_ok:
                pst[p], bad[p], done = RECEIVED_MISMATCH, j, True
                break
            if k[j] == PARENT_OTHER:
                pst[p], bad[p], done = PARENT_MISMATCH, j, True
                break
        if done:
            continue
        d = np.nonzero(k == DUPLICATE)[0]
        if d.size:
            pst[p], bad[p] = DUPLICATE_VOTE, d[0]
            continue
        yes[p] = int(choice[p * V:(p + 1) * V].astype(np.int64).sum())
        total[p] = V
    return vst, vrs, pst, bad, yes, total


def histogram(codes: np.ndarray) -> Dict[str, int]:
    c = np.bincount(codes.astype(np.int64), minlength=32)
    return {str(i): int(c[i]) for i in range(c.shape[0]) if c[i]}
