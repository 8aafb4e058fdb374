"""Struct-of-arrays packing of `Vec<Vote>` / proposals into the C-ABI layout of include/hlc.h.

A `VoteBatch` owns numpy arrays (host) that an `hlc_votes` view points into.  Fields with
variable length (owner, parent_hash, received_hash, vote_hash, signature) live in one
byte arena addressed by per-field (offset, length) pairs.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence

import numpy as np
from ctypes import c_uint8, c_uint32, c_uint64

from . import _ffi
from .protos import Proposal, Vote

FIELD_ORDER = ("vote_owner", "parent_hash", "received_hash", "vote_hash", "signature")


@dataclass
class VoteBatch:
    vote_id: np.ndarray      # u32 [n]
    proposal_id: np.ndarray  # u32 [n]
    timestamp: np.ndarray    # u64 [n]
    vote: np.ndarray         # u8  [n]
    arena: np.ndarray        # u8  [bytes]
    field_off: np.ndarray    # u64 [n, 5]
    field_len: np.ndarray    # u32 [n, 5]

    @property
    def n(self) -> int:
        return int(self.vote_id.shape[0])

    def view(self) -> _ffi.hlc_votes:
        arena = self.arena if self.arena.size else np.zeros(1, np.uint8)
        self._keep = arena
        return _ffi.hlc_votes(
            n=self.n,
            vote_id=_ffi.ptr(self.vote_id, c_uint32),
            proposal_id=_ffi.ptr(self.proposal_id, c_uint32),
            timestamp=_ffi.ptr(self.timestamp, c_uint64),
            vote=_ffi.ptr(self.vote, c_uint8),
            bytes=_ffi.ptr(arena, c_uint8),
            bytes_len=int(self.arena.size),
            field_off=_ffi.ptr(self.field_off, c_uint64),
            field_len=_ffi.ptr(self.field_len, c_uint32),
        )

    def field(self, i: int, k: int) -> bytes:
        off, ln = int(self.field_off[i, k]), int(self.field_len[i, k])
        return self.arena[off:off + ln].tobytes()

    def pinned(self) -> "VoteBatch":
        """The same batch with every array in page-locked memory (hlc_host_alloc, one
        _ffi.PinnedArena kept alive by the returned batch): hlc_validate_proposals then DMAs the
        arrays without its staging copy -- the layout an embedder that builds its batches in
        hlc_host_alloc memory hands over."""
        arrs = (self.vote_id, self.proposal_id, self.timestamp, self.vote, self.arena, self.field_off, self.field_len)
        pa = _ffi.PinnedArena(sum(a.nbytes + 64 for a in arrs) + 64)
        out = []
        for a in arrs:
            b = pa.take(a.shape, a.dtype)
            b[...] = a
            out.append(b)
        vb = VoteBatch(*out)
        vb._pinned = pa
        return vb


def pack_votes(votes: Sequence[Vote]) -> VoteBatch:
    n = len(votes)
    vote_id = np.fromiter((v.vote_id for v in votes), dtype=np.uint32, count=n)
    proposal_id = np.fromiter((v.proposal_id for v in votes), dtype=np.uint32, count=n)
    timestamp = np.fromiter((v.timestamp for v in votes), dtype=np.uint64, count=n)
    vote = np.fromiter((1 if v.vote else 0 for v in votes), dtype=np.uint8, count=n)
    field_len = np.zeros((n, 5), dtype=np.uint32)
    chunks: List[bytes] = []
    for i, v in enumerate(votes):
        for k, name in enumerate(FIELD_ORDER):
            b = getattr(v, name)
            field_len[i, k] = len(b)
            chunks.append(b)
    arena = np.frombuffer(b"".join(chunks), dtype=np.uint8).copy()
    flat = field_len.reshape(-1).astype(np.uint64)
    off = np.zeros_like(flat)
    if flat.size:
        off[1:] = np.cumsum(flat)[:-1]
    return VoteBatch(vote_id, proposal_id, timestamp, vote, arena, off.reshape(n, 5), field_len)


@dataclass
class ProposalConfig:
    """The four scalars `resolve_config` (service.rs:444-484) produces per proposal,
    minus the timeout (not on the validation path)."""
    consensus_threshold: float = 2.0 / 3.0
    max_rounds: int = 2
    use_gossipsub_rounds: bool = True


def pack_proposals(proposals: Sequence[Proposal],
                   configs: Optional[Sequence[ProposalConfig]] = None):
    """-> (VoteBatch of all votes in order, structured numpy array of hlc_proposal)."""
    votes: List[Vote] = []
    desc = np.zeros(len(proposals), dtype=_ffi.PROPOSAL_DTYPE)
    for i, p in enumerate(proposals):
        cfg = configs[i] if configs is not None else ProposalConfig()
        desc[i]["vote_begin"] = len(votes)
        desc[i]["vote_count"] = len(p.votes)
        desc[i]["proposal_id"] = p.proposal_id
        desc[i]["timestamp"] = p.timestamp
        desc[i]["expiration_timestamp"] = p.expiration_timestamp
        desc[i]["expected_voters_count"] = p.expected_voters_count
        desc[i]["max_rounds"] = cfg.max_rounds
        desc[i]["consensus_threshold"] = cfg.consensus_threshold
        desc[i]["use_gossipsub_rounds"] = 1 if cfg.use_gossipsub_rounds else 0
        desc[i]["liveness_criteria_yes"] = 1 if p.liveness_criteria_yes else 0
        votes.extend(p.votes)
    return pack_votes(votes), desc


def proposals_ptr(desc: np.ndarray):
    import ctypes
    return desc.ctypes.data_as(ctypes.POINTER(_ffi.hlc_proposal))


def results_ptr(res: np.ndarray):
    import ctypes
    return res.ctypes.data_as(ctypes.POINTER(_ffi.hlc_result))
