"""Proposal-sharded multi-GPU validation (one process per GPU, torch.distributed).

Proposals are independent on the hot path (each `process_incoming_proposal` call touches one
proposal and its votes: service.rs:263-279), so the batch shards by proposal with no data-path
collective: rank r validates proposals [bounds[r], bounds[r+1]) on its own GPU.  The only
exchange is an all_gather of the 16-byte per-proposal results (and, optionally, the 1-byte
per-vote statuses) so every rank ends with the whole batch's outcome — over RCCL on the GPU box,
gloo in the CPU tests.

`shard_bounds` splits by cumulative vote count (the work unit), not by proposal count, so ranks
stay balanced when proposal sizes differ.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

from . import _ffi
from .batch import VoteBatch


def shard_bounds(desc: np.ndarray, world: int) -> np.ndarray:
    """-> int64[world + 1] proposal-index boundaries: shard r = proposals [b[r], b[r+1]), each
    holding ~1/world of the votes (a proposal is never split)."""
    n = desc.shape[0]
    if world <= 1 or n == 0:
        return np.array([0] + [n] * max(world, 1), np.int64)
    w = np.cumsum(desc["vote_count"].astype(np.int64) + 1)  # +1: an empty proposal still costs a slot
    targets = (w[-1] * np.arange(1, world, dtype=np.float64) / world)
    cuts = np.searchsorted(w, targets, side="left") + 1
    cuts = np.minimum(np.maximum.accumulate(cuts), n)
    return np.concatenate([[0], cuts, [n]]).astype(np.int64)


def slice_shard(batch: VoteBatch, desc: np.ndarray, p0: int, p1: int) -> Tuple[VoteBatch, np.ndarray, np.ndarray]:
    """Proposals [p0, p1) with their votes as a self-contained (VoteBatch, desc) pair.
    Vote ranges are gathered (they need not be sorted), the byte arena is cut to the span the
    shard's fields use and offsets rebased.  Also returns the global index of each local vote."""
    sub = desc[p0:p1].copy()
    if sub.shape[0]:
        idx = np.concatenate([np.arange(int(d["vote_begin"]), int(d["vote_begin"]) + int(d["vote_count"]),
                                        dtype=np.int64) for d in sub])
    else:
        idx = np.zeros(0, np.int64)
    begins = np.zeros(sub.shape[0], np.uint64)
    if sub.shape[0]:
        begins[1:] = np.cumsum(sub["vote_count"].astype(np.uint64))[:-1]
    sub["vote_begin"] = begins
    off = batch.field_off[idx]
    ln = batch.field_len[idx]
    if idx.size:
        lo = int(off.min())
        hi = int((off + ln.astype(np.uint64)).max())
    else:
        lo = hi = 0
    local = VoteBatch(batch.vote_id[idx].copy(), batch.proposal_id[idx].copy(), batch.timestamp[idx].copy(),
                      batch.vote[idx].copy(), batch.arena[lo:hi].copy(), (off - np.uint64(lo)).astype(np.uint64),
                      ln.copy())
    return local, sub, idx


def _gather_rows(rows: np.ndarray, bounds: np.ndarray, rank: int, world: int, group, device) -> np.ndarray:
    """all_gather variable-length uint8 rows [count_r, width] padded to the largest shard."""
    import torch
    import torch.distributed as dist
    counts = np.diff(bounds)
    width = rows.shape[1]
    m = int(counts.max()) if counts.size else 0
    buf = torch.zeros((max(m, 1), width), dtype=torch.uint8, device=device)
    if rows.shape[0]:
        buf[:rows.shape[0]] = torch.from_numpy(np.ascontiguousarray(rows)).to(device)
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf, group=group)
    return np.concatenate([out[r][:int(counts[r])].cpu().numpy() for r in range(world)], axis=0)


def validate_sharded(engine, batch: VoteBatch, desc: np.ndarray, now: int, group=None,
                     device: Optional[str] = None, want_votes: bool = False):
    """Every rank passes the same (batch, desc); rank r validates its shard on its own engine and
    all ranks receive the full per-proposal results (and per-vote statuses if `want_votes`),
    identical to one `engine.validate_proposals` over the whole batch."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if device is None:
        device = "cpu" if dist.get_backend(group) == "gloo" else f"cuda:{__import__('torch').cuda.current_device()}"
    bounds = shard_bounds(desc, world)
    p0, p1 = int(bounds[rank]), int(bounds[rank + 1])
    local, sub, idx = slice_shard(batch, desc, p0, p1)
    res, vst, _, _ = engine.validate_proposals(local, sub, now, want_votes=want_votes)
    res = np.ascontiguousarray(res[:p1 - p0])
    rows = _gather_rows(res.view(np.uint8).reshape(-1, _ffi.RESULT_DTYPE.itemsize), bounds, rank, world, group, device)
    full = rows.reshape(-1).view(_ffi.RESULT_DTYPE).copy()
    if not want_votes:
        return full, None
    vcount = desc["vote_count"].astype(np.int64)
    vb = np.concatenate([[0], np.cumsum([int(vcount[int(bounds[r]):int(bounds[r + 1])].sum()) for r in range(world)])])
    vrows = _gather_rows(np.asarray(vst[:idx.size], np.uint8).reshape(-1, 1), vb, rank, world, group, device)
    status = np.full(batch.n, 0xFF, np.uint8)
    all_idx = np.concatenate([np.arange(int(d["vote_begin"]), int(d["vote_begin"]) + int(d["vote_count"]), dtype=np.int64)
                              for d in desc]) if desc.shape[0] else np.zeros(0, np.int64)
    status[all_idx] = vrows[:, 0]
    return full, status
