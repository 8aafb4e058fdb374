"""Deterministic synthetic signed-vote workloads, built exactly like the
reference's `build_vote` (/root/reference/src/utils.rs:55-98): each vote's received_hash is the
previous vote's hash, parent_hash is empty for distinct voters, the vote hash is SHA-256 of the
fields, and the signature is EthereumConsensusSigner::sign over the prost encoding.

Spec (frozen; tests pin the GPU generator against the CPU restatement with it):
  T0 = 1_760_000_000; proposal timestamp T0, expiration T0 + 3600, now = T0 + 1800
  vote j of a proposal: timestamp T0 + 1 + j // 1024
  global vote index i = start + p * votes_per_proposal + j
  priv(i)      = SHA256(seed_le8 || i_le8) mod n   (0 -> 1)
  vote_id(i)   = mix(seed, 2, i) | 0x80000000 (5-byte varint)
  proposal_id  = mix(seed, 1, p_global) | 0x80000000
  choice(i)    = mix(seed, 3, i) & 1
where mix is the splitmix64 finaliser of (seed*GOLDEN + domain*C2 + index) mod 2^64.

Signing / address derivation are injected (`addr_fn`, `sign_fn`) so the same generator runs on
the GPU engine (bench.py) or on the CPU restatement (tests).
"""
from __future__ import annotations

import hashlib
import struct
from dataclasses import dataclass
from typing import Callable, Optional, Tuple

import numpy as np

from . import _ffi
from .batch import VoteBatch

T0 = 1_760_000_000
EXPIRATION = T0 + 3600
NOW = T0 + 1800
N_ORDER = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
_M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
C2 = 0xD1B54A32D192ED03


def config_seed(config_no: int) -> int:
    return 0x484C4300 + config_no


def mix(seed: int, domain: int, idx: np.ndarray) -> np.ndarray:
    z = (np.uint64((seed * GOLDEN + domain * C2) & _M64) + idx.astype(np.uint64)).astype(np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def privkeys(seed: int, idx: np.ndarray) -> np.ndarray:
    out = np.zeros((idx.shape[0], 32), np.uint8)
    sb = struct.pack("<Q", seed & _M64)
    for r, i in enumerate(idx.tolist()):
        d = int.from_bytes(hashlib.sha256(sb + struct.pack("<Q", i)).digest(), "big") % N_ORDER
        if d == 0:
            d = 1
        out[r] = np.frombuffer(d.to_bytes(32, "big"), np.uint8)
    return out


def _varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


@dataclass
class Workload:
    batch: VoteBatch
    desc: np.ndarray          # hlc_proposal records
    now: int
    priv: np.ndarray          # [n, 32] signer keys (for tests that re-sign)
    name: str = ""


AddrFn = Callable[[np.ndarray], np.ndarray]
SignFn = Callable[[np.ndarray, np.ndarray, np.ndarray, np.ndarray, int], np.ndarray]


def generate(n_proposals: int, votes_per_proposal: int, expected_voters: int, gossipsub: bool, seed: int,
             addr_fn: AddrFn, sign_fn: SignFn, start_proposal: int = 0, name: str = "") -> Workload:
    """Build n_proposals chains of votes_per_proposal distinct voters each.

    sign_fn(priv[n,32], arena u8, off u64[n], len u32[n], total) -> sig[n,65] signs the payload
    slices (EIP-191 + RFC 6979 as EthereumConsensusSigner::sign)."""
    P, V = n_proposals, votes_per_proposal
    n = P * V
    p_idx = np.repeat(np.arange(P, dtype=np.uint64), V)
    j_idx = np.tile(np.arange(V, dtype=np.uint64), P)
    gidx = (np.uint64(start_proposal * V) + p_idx * np.uint64(V) + j_idx).astype(np.uint64)
    priv = privkeys(seed, gidx)
    owners = addr_fn(priv)
    pids_p = (mix(seed, 1, np.arange(start_proposal, start_proposal + P, dtype=np.uint64)) & np.uint64(0xFFFFFFFF)
              ).astype(np.uint32) | np.uint32(0x80000000)
    pid = np.repeat(pids_p, V)
    vote_id = (mix(seed, 2, gidx) & np.uint64(0xFFFFFFFF)).astype(np.uint32) | np.uint32(0x80000000)
    choice = (mix(seed, 3, gidx) & np.uint64(1)).astype(np.uint8)
    ts = (np.uint64(T0 + 1) + (j_idx // np.uint64(1024))).astype(np.uint64)

    # chained vote hashes (sequential within a proposal) and the signed payloads
    vote_hash = np.zeros((n, 32), np.uint8)
    payloads = []
    owners_b = [bytes(o) for o in owners]
    pre_h = b"\xa0\x01"
    for p in range(P):
        prev = b""
        for j in range(V):
            i = p * V + j
            vid, ppid, t, ch = int(vote_id[i]), int(pid[i]), int(ts[i]), int(choice[i])
            ob = owners_b[i]
            h = hashlib.sha256(struct.pack("<I", vid) + ob + struct.pack("<I", ppid) + struct.pack("<Q", t)
                               + bytes([ch]) + prev).digest()
            vote_hash[i] = np.frombuffer(h, np.uint8)
            enc = (pre_h + _varint(vid) + b"\xaa\x01\x14" + ob + b"\xb0\x01" + _varint(ppid) + b"\xb8\x01"
                   + _varint(t) + (b"\xc0\x01\x01" if ch else b"")
                   + ((b"\xd2\x01\x20" + prev) if prev else b"") + b"\xda\x01\x20" + h)
            payloads.append(enc)
            prev = h
    lens = np.fromiter((len(x) for x in payloads), dtype=np.uint32, count=n)
    poff = np.zeros(n, np.uint64)
    if n:
        poff[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
    parena = np.frombuffer(b"".join(payloads), np.uint8).copy()
    sig = sign_fn(priv, parena, poff, lens, int(parena.size))

    # arena per vote: owner(20) | parent(0) | received(0/32) | vote_hash(32) | sig(65)
    rec_len = np.where(j_idx > 0, 32, 0).astype(np.uint32)
    per = (20 + rec_len + 32 + 65).astype(np.uint64)
    base = np.zeros(n, np.uint64)
    if n:
        base[1:] = np.cumsum(per)[:-1]
    arena = np.zeros(int(per.sum()), np.uint8)
    field_off = np.zeros((n, 5), np.uint64)
    field_len = np.zeros((n, 5), np.uint32)
    field_len[:, 0] = 20
    field_len[:, 2] = rec_len
    field_len[:, 3] = 32
    field_len[:, 4] = 65
    field_off[:, 0] = base
    field_off[:, 1] = base + 20
    field_off[:, 2] = base + 20
    field_off[:, 3] = base + 20 + rec_len
    field_off[:, 4] = base + 20 + rec_len + 32
    # vectorised scatter of the fixed-size fields
    for k, src, width in ((0, owners, 20), (3, vote_hash, 32), (4, sig, 65)):
        idx = field_off[:, k][:, None] + np.arange(width, dtype=np.uint64)[None, :]
        arena[idx.reshape(-1)] = src.reshape(-1)
    has_rec = j_idx > 0
    if has_rec.any():
        prev_hash = np.roll(vote_hash, 1, axis=0)
        idx = field_off[has_rec, 2][:, None] + np.arange(32, dtype=np.uint64)[None, :]
        arena[idx.reshape(-1)] = prev_hash[has_rec].reshape(-1)

    batch = VoteBatch(vote_id=vote_id, proposal_id=pid, timestamp=ts, vote=choice, arena=arena,
                      field_off=field_off, field_len=field_len)
    desc = np.zeros(P, dtype=_ffi.PROPOSAL_DTYPE)
    desc["vote_begin"] = np.arange(P, dtype=np.uint64) * np.uint64(V)
    desc["vote_count"] = V
    desc["proposal_id"] = pids_p
    desc["timestamp"] = T0
    desc["expiration_timestamp"] = EXPIRATION
    desc["expected_voters_count"] = expected_voters
    desc["max_rounds"] = 2 if gossipsub else 0
    desc["consensus_threshold"] = 2.0 / 3.0
    desc["use_gossipsub_rounds"] = 1 if gossipsub else 0
    desc["liveness_criteria_yes"] = 1
    return Workload(batch, desc, NOW, priv, name)


def engine_signers(engine) -> Tuple[AddrFn, SignFn]:
    """(addr_fn, sign_fn) backed by the GPU engine."""
    def addr_fn(priv):
        return engine.address_batch(priv)

    def sign_fn(priv, arena, off, lens, total):
        return engine.sign_batch_arena(priv, arena, off, lens, total)

    return addr_fn, sign_fn


def to_wire(batch: VoteBatch, desc: np.ndarray, names=None):
    """Encode the proposals of a (batch, desc) workload as gossip bytes: one prost `Proposal`
    message (consensus.proto:5-16, votes included with their signatures) per proposal,
    concatenated.  Returns (wire u8[bytes], msg_off u64[P], msg_len u32[P], scope
    SCOPE_CONFIG_DTYPE[P]) -- the inputs of hlc_validate_wire_proposals."""
    def vbytes(i: int) -> bytes:
        out = bytearray()
        vid, pid, ts = int(batch.vote_id[i]), int(batch.proposal_id[i]), int(batch.timestamp[i])
        if vid:
            out += b"\xa0\x01" + _varint(vid)
        fo, fl = batch.field_off[i], batch.field_len[i]
        arena = batch.arena

        def fld(k):
            return arena[int(fo[k]):int(fo[k]) + int(fl[k])].tobytes()
        if fl[0]:
            out += b"\xaa\x01" + _varint(int(fl[0])) + fld(0)
        if pid:
            out += b"\xb0\x01" + _varint(pid)
        if ts:
            out += b"\xb8\x01" + _varint(ts)
        if batch.vote[i]:
            out += b"\xc0\x01\x01"
        for k, key in ((1, b"\xca\x01"), (2, b"\xd2\x01"), (3, b"\xda\x01"), (4, b"\xe2\x01")):
            if fl[k]:
                out += key + _varint(int(fl[k])) + fld(k)
        return bytes(out)

    msgs = []
    for p in range(desc.shape[0]):
        d = desc[p]
        out = bytearray()
        name = (names[p] if names is not None else f"proposal-{p}").encode()
        if name:
            out += b"\x52" + _varint(len(name)) + name
        if int(d["proposal_id"]):
            out += b"\x60" + _varint(int(d["proposal_id"]))
        b0, cnt = int(d["vote_begin"]), int(d["vote_count"])
        for i in range(b0, b0 + cnt):
            ev = vbytes(i)
            out += b"\x72" + _varint(len(ev)) + ev
        for key, val in ((b"\x78", int(d["expected_voters_count"])), (b"\x80\x01", 1),
                         (b"\x88\x01", int(d["timestamp"])), (b"\x90\x01", int(d["expiration_timestamp"]))):
            if val:
                out += key + _varint(val)
        if d["liveness_criteria_yes"]:
            out += b"\x98\x01\x01"
        msgs.append(bytes(out))
    lens = np.fromiter((len(m) for m in msgs), dtype=np.uint32, count=len(msgs))
    off = np.zeros(len(msgs), np.uint64)
    if msgs:
        off[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
    wire = np.frombuffer(b"".join(msgs), np.uint8).copy()
    scope = np.zeros(desc.shape[0], _ffi.SCOPE_CONFIG_DTYPE)
    scope["consensus_threshold"] = desc["consensus_threshold"]
    scope["max_rounds"] = desc["max_rounds"]
    scope["use_gossipsub_rounds"] = desc["use_gossipsub_rounds"]
    return wire, off, lens, scope
