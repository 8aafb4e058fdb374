"""a config-2-shaped workload with ~1/3 Byzantine votes, split evenly
over the mutation kinds below, built with the CPU restatements (test infrastructure).

Mutation kinds (expected first outcome in brackets):
  wrong_key     signed by another key                        [InvalidVoteSignature]
  flip_rs       one bit of r or s flipped                     [InvalidVoteSignature / scheme]
  bad_v         v in {2, 29, 34}                               [SignatureScheme: parity]
  high_s        s -> n - s, parity flipped (still valid)      [Ok]
  no_point      r with x^3+7 a non-residue                    [SignatureScheme: no point]
  infinity      crafted R = kG, s = z/k  =>  Q = infinity     [SignatureScheme: infinity]
  tamper_hash   vote_hash bit flipped                         [InvalidVoteHash]
  bad_received  received_hash replaced, vote re-hashed+signed [ReceivedHashMismatch]
  parent_other  parent_hash -> another owner's vote, re-signed [ParentHashMismatch]
  ts_regress    timestamp below the previous vote, re-signed  [ReceivedHashMismatch]
  ts_old        timestamp before proposal creation, re-signed [TimestampOlderThanCreationTime]
  duplicate     a second vote by an earlier voter, re-signed  [DuplicateVote]
  wrong_pid     proposal_id changed, re-signed                [VoteProposalIdMismatch]
  empty         owner / vote_hash / signature emptied         [Empty*]
  sig_len       signature truncated / extended                [SignatureScheme: length]
"""
from __future__ import annotations

import random
from typing import List, Tuple

import numpy as np

import coracle
import pyoracle as po
from hashgraph_like_consensus.batch import pack_votes

KINDS = ["wrong_key", "flip_rs", "bad_v", "high_s", "no_point", "infinity", "tamper_hash", "bad_received",
         "parent_other", "ts_regress", "ts_old", "duplicate", "wrong_pid", "empty", "sig_len"]


def batch_to_votes(batch, lo: int = 0, hi: int = -1) -> List[po.Vote]:
    out = []
    for i in range(lo, batch.n if hi < 0 else hi):
        f = [batch.field(i, k) for k in range(5)]
        out.append(po.Vote(vote_id=int(batch.vote_id[i]), vote_owner=f[0], proposal_id=int(batch.proposal_id[i]),
                           timestamp=int(batch.timestamp[i]), vote=bool(batch.vote[i]), parent_hash=f[1],
                           received_hash=f[2], vote_hash=f[3], signature=f[4]))
    return out


def c_sign(priv: int, v: po.Vote) -> bytes:
    h = coracle.eip191_hash(po.signed_payload(v))
    key = np.frombuffer(priv.to_bytes(32, "big"), np.uint8).reshape(1, 32)
    return coracle.sign_batch(key, np.frombuffer(h, np.uint8).reshape(1, 32), 1)[0].tobytes()


def resign(v: po.Vote, priv: int, rehash: bool = True) -> None:
    if rehash:
        v.vote_hash = po.compute_vote_hash(v)
    v.signature = b""
    v.signature = c_sign(priv, v)


class _Deferred:
    """Deferred signing for the mutation pass.  A signature never feeds a vote hash or a signed
    payload (utils.rs:37-47, 150-152), so every re-sign only records (payload snapshot, key) and
    one multithreaded C-oracle pass signs them all at the end; signature-level mutations (which
    read the signature) are queued and applied after it, in order.  The output is byte-identical
    to signing immediately (tests/test_adversarial_fast.py)."""

    def __init__(self):
        self.pending = {}   # vote index -> (payload, priv)
        self.sig_ops = []   # (vote index, op, args) in mutation order

    def resign(self, votes, i: int, priv: int, rehash: bool = True) -> None:
        v = votes[i]
        if rehash:
            v.vote_hash = po.compute_vote_hash(v)
        v.signature = b""
        self.pending[i] = (po.signed_payload(v), priv)

    def sign_other(self, votes, i: int, priv: int) -> None:
        self.pending[i] = (po.signed_payload(votes[i]), priv)

    def flush(self, votes, threads: int = 16, sign_payloads=None) -> None:
        """sign_payloads(keys u8[m,32], payloads) -> sig u8[m,65] (e.g. the GPU engine's
        sign_batch); default: the C oracle."""
        idx = list(self.pending)
        if idx:
            keys = np.stack([np.frombuffer(self.pending[i][1].to_bytes(32, "big"), np.uint8) for i in idx])
            if sign_payloads is not None:
                sigs = sign_payloads(keys, [self.pending[i][0] for i in idx])
            else:
                pre = np.stack([np.frombuffer(coracle.eip191_hash(self.pending[i][0]), np.uint8) for i in idx])
                sigs = coracle.sign_batch(keys, pre, threads=threads)
            for k, i in enumerate(idx):
                votes[i].signature = sigs[k].tobytes()
        for i, op, arg in self.sig_ops:
            v = votes[i]
            s = bytearray(v.signature)
            if op == "xor":
                s[arg[0]] ^= arg[1]
            elif op == "v":
                s[64] = arg
            elif op == "high_s":
                sv = int.from_bytes(s[32:64], "big")
                s[32:64] = (po.N - sv).to_bytes(32, "big")
                s[64] = 55 - s[64]
            elif op == "r":
                s[0:32] = arg
            elif op == "set":
                s = bytearray(arg)
            elif op == "trunc":
                s = s[:64] if arg else s + b"\x00"
            v.signature = bytes(s)


_NO_POINT_R = None


def no_point_r() -> int:
    global _NO_POINT_R
    if _NO_POINT_R is None:
        r = 2**255 + 12345
        while po.decompress(r, False) is not None:
            r += 1
        _NO_POINT_R = r
    return _NO_POINT_R


def relink_after(votes: List[po.Vote], privs: List[int], i: int, end: int, dfr: "_Deferred") -> None:
    """Re-chain votes i+1 .. end-1 after vote i's hash changed: received_hash -> previous vote,
    then re-hash and re-sign, so the chain stays valid (the mutation's own class surfaces)."""
    for k in range(i + 1, end):
        votes[k].received_hash = votes[k - 1].vote_hash
        dfr.resign(votes, k, privs[k])


def _kg(k: int):
    from crypto_items import _kg as kg
    return kg(k)


def mutate(votes: List[po.Vote], privs: List[int], i: int, j: int, kind: str, rnd: random.Random,
           begin: int, end: int = 0, dfr: "_Deferred" = None) -> None:
    """Mutate votes[i] (index j within its proposal [begin, end)).  Signing is deferred to
    dfr.flush() (see _Deferred)."""
    own = dfr is None
    if own:
        dfr = _Deferred()
    v = votes[i]
    priv = privs[i]
    if kind == "wrong_key":
        dfr.sign_other(votes, i, rnd.randrange(1, po.N))
    elif kind == "flip_rs":
        pos = rnd.randrange(64)
        dfr.sig_ops.append((i, "xor", (pos, 1 << rnd.randrange(8))))
    elif kind == "bad_v":
        dfr.sig_ops.append((i, "v", rnd.choice([2, 29, 34])))
    elif kind == "high_s":
        dfr.sig_ops.append((i, "high_s", None))
    elif kind == "no_point":
        dfr.sig_ops.append((i, "r", no_point_r().to_bytes(32, "big")))
    elif kind == "infinity":
        z = int.from_bytes(coracle.eip191_hash(po.signed_payload(v)), "big") % po.N
        k = rnd.randrange(1, po.N)
        rx, ry = _kg(k)
        r = rx % po.N
        s = z * pow(k, -1, po.N) % po.N
        if s == 0:
            s = 1
        dfr.sig_ops.append((i, "set", r.to_bytes(32, "big") + s.to_bytes(32, "big") + bytes([27 + (ry & 1)])))
    elif kind == "tamper_hash":
        h = bytearray(v.vote_hash)
        h[rnd.randrange(32)] ^= 0x10
        v.vote_hash = bytes(h)
    elif kind == "bad_received":
        v.received_hash = bytes(rnd.randrange(256) for _ in range(32))
        dfr.resign(votes, i, priv)
    elif kind == "parent_other":
        if j >= 2:
            other = votes[begin + rnd.randrange(j - 1)]
            v.parent_hash = other.vote_hash
        else:
            v.parent_hash = bytes(32)
        dfr.resign(votes, i, priv)
    elif kind == "ts_regress":
        v.timestamp = max(votes[i - 1].timestamp - 1, 0) if j > 0 else v.timestamp
        dfr.resign(votes, i, priv)
    elif kind == "ts_old":
        v.timestamp = v.timestamp - 10_000
        dfr.resign(votes, i, priv)
    elif kind == "duplicate":
        if j >= 1:
            src = begin + rnd.randrange(j)
            v.vote_owner = votes[src].vote_owner
            privs[i] = privs[src]
            dfr.resign(votes, i, privs[i])
            relink_after(votes, privs, i, end, dfr)
    elif kind == "wrong_pid":
        v.proposal_id = (v.proposal_id + 1) & 0xFFFFFFFF
        dfr.resign(votes, i, priv)
    elif kind == "empty":
        which = rnd.randrange(3)
        if which == 0:
            v.vote_owner = b""
        elif which == 1:
            v.vote_hash = b""
        else:
            dfr.sig_ops.append((i, "set", b""))
    elif kind == "sig_len":
        dfr.sig_ops.append((i, "trunc", rnd.random() < 0.5))
    else:
        raise ValueError(kind)
    if own:
        dfr.flush(votes, threads=1)


def byzantine(workload, fraction: float = 1 / 3, seed: int = 5, kinds_pool=None,
              sign_payloads=None) -> Tuple[object, np.ndarray, List[str]]:
    """-> (VoteBatch with mutations, desc, per-vote kind or '').  kinds_pool restricts the kinds;
    sign_payloads: the re-signing backend (see _Deferred.flush)."""
    pool = list(kinds_pool) if kinds_pool else KINDS
    rnd = random.Random(seed)
    votes = batch_to_votes(workload.batch)
    privs = [int.from_bytes(bytes(k), "big") for k in workload.priv]
    kinds = [""] * len(votes)
    desc = workload.desc
    dfr = _Deferred()
    k = 0
    for p in range(desc.shape[0]):
        b, c = int(desc[p]["vote_begin"]), int(desc[p]["vote_count"])
        for j in range(c):
            if rnd.random() < fraction:
                kind = pool[k % len(pool)]
                k += 1
                mutate(votes, privs, b + j, j, kind, rnd, b, b + c, dfr)
                kinds[b + j] = kind
    dfr.flush(votes, threads=max(1, min(16, __import__("os").cpu_count() or 1)), sign_payloads=sign_payloads)
    return pack_votes(votes), desc, kinds


def proposals_from_batch(batch, desc) -> List[po.Proposal]:
    votes = batch_to_votes(batch)
    out = []
    for d in desc:
        b, c = int(d["vote_begin"]), int(d["vote_count"])
        out.append(po.Proposal(proposal_id=int(d["proposal_id"]), votes=votes[b:b + c],
                               expected_voters_count=int(d["expected_voters_count"]), timestamp=int(d["timestamp"]),
                               expiration_timestamp=int(d["expiration_timestamp"]),
                               liveness_criteria_yes=bool(d["liveness_criteria_yes"])))
    return out


def config_of(d) -> po.ConsensusConfig:
    return po.ConsensusConfig(float(d["consensus_threshold"]), int(d["max_rounds"]), bool(d["use_gossipsub_rounds"]),
                              bool(d["liveness_criteria_yes"]))
