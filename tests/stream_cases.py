"""Streaming-vote workloads (process_incoming_vote micro-batches) shared by the CPU and GPU tests."""
from __future__ import annotations

import random
from typing import List, Tuple

import numpy as np

import pyoracle as po
import stream_oracle as so
from adversarial import batch_to_votes, byzantine
from hashgraph_like_consensus import _ffi
from hashgraph_like_consensus.batch import pack_votes
from helpers import oracle_workload


def sessions_array(sessions: List[so.Session]) -> np.ndarray:
    a = np.zeros(len(sessions), _ffi.SESSION_DTYPE)
    for k, s in enumerate(sessions):
        a[k] = (s.timestamp, s.expiration_timestamp, s.proposal_id, s.expected_voters_count, s.round, s.total, s.yes,
                s.max_rounds, s.consensus_threshold, s.state, int(s.use_gossipsub_rounds),
                int(s.liveness_criteria_yes), (0,) * 5)
    return a


def owners_arrays(sessions: List[so.Session]) -> Tuple[np.ndarray, np.ndarray]:
    rows, sess = [], []
    for k, s in enumerate(sessions):
        for o in sorted(s.owners):
            rows.append(np.frombuffer(o, np.uint8))
            sess.append(k)
    if not rows:
        return np.zeros((0, 20), np.uint8), np.zeros(0, np.uint32)
    return np.stack(rows), np.array(sess, np.uint32)


def streaming_workload(seed: int, n_props: int = 24, votes: int = 12, p2p_every: int = 4):
    """-> (sessions, votes (po.Vote), vote_session, now): sessions built from a signed workload,
    some pre-populated with the first votes of their chain, some already decided / Failed / at
    their expiry; then the remaining votes delivered shuffled across sessions, with replays
    (duplicates), Byzantine mutations and votes for unknown sessions mixed in."""
    rnd = random.Random(seed)
    w = oracle_workload(n_props, votes, votes, True, seed, name=f"stream-{seed}")
    bbatch, desc, kinds = byzantine(w, fraction=1 / 5, seed=seed + 1)
    allv = batch_to_votes(bbatch)
    clean = batch_to_votes(w.batch)
    now = w.now
    sessions: List[so.Session] = []
    deliveries = []
    for p in range(n_props):
        d = desc[p]
        b, c = int(d["vote_begin"]), int(d["vote_count"])
        gossip = p % p2p_every != 0
        s = so.Session(proposal_id=int(d["proposal_id"]), timestamp=int(d["timestamp"]),
                       expiration_timestamp=int(d["expiration_timestamp"]),
                       expected_voters_count=int(d["expected_voters_count"]) + rnd.choice([0, 0, 3]),
                       round=1, total=0, yes=0, max_rounds=2 if gossip else rnd.choice([0, 0, 5, 9]),
                       consensus_threshold=rnd.choice([2.0 / 3.0, 2.0 / 3.0, 0.5, 0.9]),
                       state=po.SESSION_ACTIVE, use_gossipsub_rounds=gossip,
                       liveness_criteria_yes=rnd.random() < 0.7)
        pre = rnd.choice([0, 0, 1, 3])                     # votes already in the session's map
        for j in range(pre):
            v = clean[b + j]
            s.owners.add(v.vote_owner)
            s.total += 1
            s.yes += 1 if v.vote else 0
            s.round = 2 if gossip else s.round + 1
        kind = rnd.random()
        if kind < 0.08:
            s.state = po.SESSION_REACHED_YES
        elif kind < 0.14:
            s.state = po.SESSION_FAILED
        elif kind < 0.2:
            s.expiration_timestamp = now                    # validate_vote passes, add_vote: ProposalExpired
        sessions.append(s)
        for j in range(pre, c):
            deliveries.append((allv[b + j], p))
            if rnd.random() < 0.1:
                deliveries.append((allv[b + j], p))     # replay: DuplicateVote if the first was inserted
    rnd.shuffle(deliveries)
    # votes whose session does not exist (storage miss)
    for _ in range(5):
        v, _p = deliveries[rnd.randrange(len(deliveries))]
        deliveries.insert(rnd.randrange(len(deliveries)), (v, -1))
    # a vote mapped to a session of another proposal (caller error -> id mismatch)
    v, p = deliveries[0]
    deliveries.append((v, (p + 1) % n_props))
    votes_ = [v for v, _ in deliveries]
    vs = [p for _, p in deliveries]
    return sessions, votes_, vs, now


def run_oracle(sessions, votes_, vs, now):
    import copy
    ss = copy.deepcopy(sessions)
    out = so.process_incoming_votes(ss, votes_, vs, now)
    return ss, out


def device_inputs(sessions, votes_, vs):
    batch = pack_votes(votes_)
    vsess = np.array([0xFFFFFFFF if p < 0 else p for p in vs], np.uint32)
    owners, osess = owners_arrays(sessions)
    return batch, vsess, sessions_array(sessions), owners, osess
