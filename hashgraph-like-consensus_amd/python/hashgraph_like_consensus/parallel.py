"""Proposal-sharded multi-GPU validation (one process per GPU, torch.distributed).

Proposals are independent on the hot path (each `process_incoming_proposal` call touches one
proposal and its votes: service.rs:263-279), so the batch shards by proposal with no data-path
collective: rank r validates proposals [bounds[r], bounds[r+1]) on its own GPU.  The only
exchange is an all_gather of the 16-byte per-proposal results (and, optionally, the 1-byte
per-vote statuses) so every rank ends with the whole batch's outcome — over RCCL on the GPU box,
gloo in the CPU tests.

`shard_bounds` splits by cumulative vote count (the work unit), not by proposal count, so ranks
stay balanced when proposal sizes differ.

The two other entry paths shard the same way: `validate_wire_sharded` gives each
rank a byte-balanced range of gossip messages (decode + validation on its GPU), and
`process_votes_sharded` places session s on rank s % world, so every incoming vote is processed
by the rank holding its session's state -- again with only the results gathered.
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


N_CODES = 32  # status histogram width (HLC_* codes are < 32)


class ShardExchange:
    """The one exchange step of a proposal-sharded run, device-resident: every
    rank's 16-byte per-proposal results are all-gathered (padded to the largest shard) and the
    outcome counters -- a histogram of per-vote statuses (code 0 = verified) and one of
    per-proposal statuses -- are all-reduced (sum).  Over RCCL on GPUs (bench.py), gloo on CPU
    tensors in the tests.  Nothing else crosses ranks: every check is intra-proposal."""

    def __init__(self, max_proposals: int, world: int, device, group=None, engine=None):
        import torch
        self.torch = torch
        self.engine = engine  # device tensors: the engine's counter kernel (hlc_outcome_counts_device)
        self.group = group
        self.world = world
        self.max_p = int(max_proposals)
        self.send = torch.zeros(max(self.max_p, 1) * 16, dtype=torch.uint8, device=device)
        self.rows = torch.empty(world * max(self.max_p, 1) * 16, dtype=torch.uint8, device=device)
        self.counters = torch.zeros(2 * N_CODES, dtype=torch.int64, device=device)

    def local_counters(self, results_u8, status_u8, n_props: int, n_votes: int) -> None:
        """Fixed-width histograms with no host read-back (a torch.bincount reads max/min back and
        synchronises the host every step).  On the GPU: the engine's counter kernel, an LDS
        histogram per block on the current stream (a scatter_add_ of 640k all-OK votes into one bin
        serialised on one address: 80 us per call).  On CPU tensors (the gloo tests): scatter_add_.
        Every HLC_* code is < N_CODES; a larger byte is counted in the last bin."""
        t = self.torch
        c = self.counters
        if self.engine is not None and c.is_cuda:
            self.engine.outcome_counts_device(status_u8.data_ptr(), n_votes, results_u8.data_ptr(), n_props,
                                              c.data_ptr(), t.cuda.current_stream(c.device).cuda_stream)
            return
        c.zero_()
        sv = status_u8[:n_votes].long().clamp_(max=N_CODES - 1)
        c[:N_CODES].scatter_add_(0, sv, t.ones_like(sv))
        pv = results_u8[: n_props * 16].view(-1, 16)[:, 0].long().clamp_(max=N_CODES - 1)
        c[N_CODES:].scatter_add_(0, pv, t.ones_like(pv))

    def __call__(self, results_u8, status_u8, n_props: int, n_votes: int) -> None:
        import torch.distributed as dist
        self.local_counters(results_u8, status_u8, n_props, n_votes)
        self.send[: n_props * 16].copy_(results_u8[: n_props * 16])
        if n_props < self.max_p:
            self.send[n_props * 16:].zero_()
        dist.all_gather_into_tensor(self.rows, self.send, group=self.group)
        dist.all_reduce(self.counters, group=self.group)

    def results(self, counts) -> np.ndarray:
        """The gathered results of every rank in rank order (counts[r] = rank r's proposals)."""
        rows = self.rows.cpu().numpy().reshape(self.world, -1)
        return np.concatenate([rows[r, : int(counts[r]) * 16] for r in range(self.world)]).view(_ffi.RESULT_DTYPE)

    def summary(self) -> dict:
        c = self.counters.cpu().numpy()
        return {"verified_votes": int(c[0]),
                "rejected_votes_by_status": {str(k): int(c[k]) for k in range(1, N_CODES) if c[k]},
                "proposals_ok": int(c[N_CODES]),
                "proposals_by_status": {str(k): int(c[N_CODES + k]) for k in range(1, N_CODES) if c[N_CODES + k]}}


def validate_shard(engine, local: VoteBatch, local_desc: np.ndarray, now: int, group=None,
                   device: Optional[str] = None, want_votes: bool = False):
    """Each rank passes ONLY its own shard (its proposals and their votes, generated or loaded by
    that rank) and receives every rank's per-proposal results in rank order, the all-reduced
    outcome counters, and (want_votes) every rank's per-vote statuses in rank order."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if device is None:
        device = "cpu" if dist.get_backend(group) == "gloo" else f"cuda:{torch.cuda.current_device()}"
    P = int(local_desc.shape[0])
    n = int(local_desc["vote_count"].astype(np.int64).sum()) if P else 0
    res, vst, _, _ = engine.validate_proposals(local, local_desc, now, want_votes=True)
    sizes = torch.tensor([P, n], dtype=torch.int64, device=device)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    counts = np.array([int(x[0]) for x in all_sizes], np.int64)
    vcounts = np.array([int(x[1]) for x in all_sizes], np.int64)
    ex = ShardExchange(int(counts.max()) if counts.size else 0, world, device, group)
    res_t = torch.from_numpy(np.ascontiguousarray(res[:P]).view(np.uint8).reshape(-1).copy()).to(device)
    # per-vote statuses of the proposals' votes, in proposal order
    idx = np.concatenate([np.arange(int(d["vote_begin"]), int(d["vote_begin"]) + int(d["vote_count"]),
                                    dtype=np.int64) for d in local_desc]) if P else np.zeros(0, np.int64)
    st_local = np.asarray(vst, np.uint8)[idx] if idx.size else np.zeros(0, np.uint8)
    st_t = torch.from_numpy(st_local.copy()).to(device)
    ex(res_t, st_t, P, n)
    full = ex.results(counts).copy()
    if not want_votes:
        return full, None, ex.summary()
    vb = np.concatenate([[0], np.cumsum(vcounts)])
    vrows = _gather_rows(st_local.reshape(-1, 1), vb, dist.get_rank(group), world, group, device)
    return full, vrows[:, 0].copy(), ex.summary()


def validate_sharded(engine, batch: VoteBatch, desc: np.ndarray, now: int, group=None,
                     device: Optional[str] = None, want_votes: bool = False):
    """Convenience over validate_shard when every rank holds the same (batch, desc): rank r cuts
    its shard out and validates only that; all ranks receive the full per-proposal results (and
    per-vote statuses if `want_votes`), identical to one `engine.validate_proposals` over the
    whole batch.  At scale, generate or load only the rank's shard and call validate_shard."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    bounds = shard_bounds(desc, world)
    p0, p1 = int(bounds[rank]), int(bounds[rank + 1])
    local, sub, _ = slice_shard(batch, desc, p0, p1)
    full, vst, _ = validate_shard(engine, local, sub, now, group, device, want_votes)
    if not want_votes:
        return full, None
    status = np.full(batch.n, 0xFF, np.uint8)
    all_idx = np.concatenate([np.arange(int(d["vote_begin"]), int(d["vote_begin"]) + int(d["vote_count"]), dtype=np.int64)
                              for d in desc]) if desc.shape[0] else np.zeros(0, np.int64)
    status[all_idx] = vst
    return full, status


# ---- wire path: messages are independent proposals -------------------------------------------
def wire_shard_bounds(msg_len: np.ndarray, world: int) -> np.ndarray:
    """-> int64[world + 1] message-index boundaries holding ~1/world of the wire bytes each (the
    bytes track the vote count, the work unit)."""
    n = int(msg_len.shape[0])
    if world <= 1 or n == 0:
        return np.array([0] + [n] * max(world, 1), np.int64)
    w = np.cumsum(msg_len.astype(np.int64) + 1)
    cuts = np.searchsorted(w, w[-1] * np.arange(1, world, dtype=np.float64) / world, side="left") + 1
    cuts = np.minimum(np.maximum.accumulate(cuts), n)
    return np.concatenate([[0], cuts, [n]]).astype(np.int64)


def validate_wire_sharded(engine, wire: np.ndarray, msg_off: np.ndarray, msg_len: np.ndarray, scope: np.ndarray,
                          now: int, group=None, device: Optional[str] = None):
    """Every rank passes the same gossip bytes; rank r decodes + validates its contiguous range of
    messages (hlc_validate_wire_proposals on its own GPU) and all ranks receive every message's
    (hlc_result, hlc_wire_proposal), identical to one call over the whole batch."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if device is None:
        device = "cpu" if dist.get_backend(group) == "gloo" else f"cuda:{__import__('torch').cuda.current_device()}"
    bounds = wire_shard_bounds(msg_len, world)
    m0, m1 = int(bounds[rank]), int(bounds[rank + 1])
    sc = scope if scope.shape[0] == 1 else scope[m0:m1]
    if m1 > m0:
        lo = int(msg_off[m0:m1].min())
        hi = int((msg_off[m0:m1] + msg_len[m0:m1].astype(np.uint64)).max())
        res, winfo, _ = engine.validate_wire_proposals(wire[lo:hi], msg_off[m0:m1] - np.uint64(lo), msg_len[m0:m1],
                                                       sc, now)
    else:
        res = np.zeros(0, _ffi.RESULT_DTYPE)
        winfo = np.zeros(0, _ffi.WIRE_PROPOSAL_DTYPE)
    rrows = _gather_rows(np.ascontiguousarray(res).view(np.uint8).reshape(-1, _ffi.RESULT_DTYPE.itemsize), bounds,
                         rank, world, group, device)
    wrows = _gather_rows(np.ascontiguousarray(winfo).view(np.uint8).reshape(-1, _ffi.WIRE_PROPOSAL_DTYPE.itemsize),
                         bounds, rank, world, group, device)
    return (rrows.reshape(-1).view(_ffi.RESULT_DTYPE).copy(), wrows.reshape(-1).view(_ffi.WIRE_PROPOSAL_DTYPE).copy())


# ---- streaming path: sessions are independent --------------------------------------------------
def process_votes_sharded(engine, batch: VoteBatch, vote_session: np.ndarray, sessions: np.ndarray,
                          owners: np.ndarray, owner_session: np.ndarray, now: int, group=None,
                          device: Optional[str] = None):
    """Micro-batched process_incoming_vote across ranks: session s lives on rank s % world (its
    owner map with it), so each rank processes exactly the votes of its sessions, in delivery
    order, on its own GPU (hlc_process_votes) -- no vote ever needs another rank's state.  Every
    rank passes the same inputs and receives every vote's (status, transition, inserted, reason)
    and every session's final state, identical to one call over the whole batch."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if device is None:
        device = "cpu" if dist.get_backend(group) == "gloo" else f"cuda:{__import__('torch').cuda.current_device()}"
    S = sessions.shape[0]
    mine_s = np.arange(rank, S, world, dtype=np.int64)              # my sessions (global ids)
    local_of = np.full(S, 0xFFFFFFFF, np.int64)
    local_of[mine_s] = np.arange(mine_s.size)
    vs = vote_session.astype(np.int64)
    found = vs != 0xFFFFFFFF
    vsafe = np.where(found, vs, 0)
    # votes for missing sessions are answered by rank 0 (SessionNotFound needs no state)
    mine_v = np.nonzero(np.where(found, (vsafe % world) == rank, rank == 0))[0]
    sub = VoteBatch(batch.vote_id[mine_v], batch.proposal_id[mine_v], batch.timestamp[mine_v], batch.vote[mine_v],
                    batch.arena, batch.field_off[mine_v], batch.field_len[mine_v])
    lvs = np.where(found[mine_v], local_of[vsafe[mine_v]], 0xFFFFFFFF).astype(np.uint32)
    lsess = np.ascontiguousarray(sessions[mine_s])
    omask = (owner_session.astype(np.int64) % world) == rank
    lown = np.ascontiguousarray(owners[omask]).reshape(-1, 20)
    losess = local_of[owner_session[omask].astype(np.int64)].astype(np.uint32)
    st, tr, ins, rs = engine.process_votes(sub, lvs, lsess, lown, losess, now)
    # gather per-vote outputs (rows: global index u64 + 4 bytes) and session rows
    vrow = np.zeros((mine_v.size, 12), np.uint8)
    vrow[:, :8] = mine_v.astype(np.uint64).view(np.uint8).reshape(-1, 8)
    vrow[:, 8], vrow[:, 9], vrow[:, 10], vrow[:, 11] = st, tr, ins, rs
    import torch
    counts = torch.tensor([mine_v.size, mine_s.size], dtype=torch.int64, device=device)
    allc = [torch.zeros_like(counts) for _ in range(world)]
    dist.all_gather(allc, counts, group=group)
    vb = np.concatenate([[0], np.cumsum([int(c[0]) for c in allc])])
    sb = np.concatenate([[0], np.cumsum([int(c[1]) for c in allc])])
    vrows = _gather_rows(vrow, vb, rank, world, group, device)
    srow = np.zeros((mine_s.size, 8 + _ffi.SESSION_DTYPE.itemsize), np.uint8)
    srow[:, :8] = mine_s.astype(np.uint64).view(np.uint8).reshape(-1, 8)
    srow[:, 8:] = lsess.view(np.uint8).reshape(-1, _ffi.SESSION_DTYPE.itemsize)
    srows = _gather_rows(srow, sb, rank, world, group, device)
    n = batch.n
    out = np.zeros((4, n), np.uint8)
    gi = vrows[:, :8].copy().view(np.uint64).reshape(-1).astype(np.int64)
    out[:, gi] = vrows[:, 8:12].T
    final = sessions.copy()
    si = srows[:, :8].copy().view(np.uint64).reshape(-1).astype(np.int64)
    final[si] = srows[:, 8:].copy().reshape(-1).view(_ffi.SESSION_DTYPE)
    return out[0], out[1], out[2], out[3], final
