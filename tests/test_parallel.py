"""Proposal-sharded multi-process path (parallel.py) on CPU: gloo, world size 2.

Each rank validates its shard with an oracle-backed engine double (test infrastructure) and the
gathered results must equal one whole-batch validation.  The same code runs over RCCL on GPUs
(bench.py's N > 1 path shards the same way).
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import coracle
from adversarial import byzantine
from helpers import oracle_workload
from hashgraph_like_consensus.parallel import shard_bounds, slice_shard


class OracleEngine:
    def validate_proposals(self, batch, desc, now, want_votes=True, want_recovered=False):
        return coracle.validate_proposals(batch, desc, now, threads=2)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_bounds_balanced_and_total():
    desc = np.zeros(10, dtype=__import__("hashgraph_like_consensus._ffi", fromlist=["x"]).PROPOSAL_DTYPE)
    desc["vote_count"] = [100, 1, 1, 1, 1, 1, 1, 1, 1, 100]
    b = shard_bounds(desc, 2)
    assert b[0] == 0 and b[-1] == 10 and np.all(np.diff(b) >= 0)
    w = [int(desc["vote_count"][b[r]:b[r + 1]].sum()) for r in range(2)]
    assert abs(w[0] - w[1]) <= 100
    assert list(shard_bounds(desc, 1)) == [0, 10]
    b16 = shard_bounds(desc, 16)
    assert len(b16) == 17 and b16[-1] == 10 and np.all(np.diff(b16) >= 0)
    empty = desc[:0]
    assert list(shard_bounds(empty, 4)) == [0, 0, 0, 0, 0]


def test_slice_shard_equals_whole_batch():
    w = oracle_workload(6, 5, 8, True, seed=41)
    batch, desc, _ = byzantine(w, fraction=0.3, seed=3)
    ref, vst_ref, _, _ = coracle.validate_proposals(batch, desc, w.now, threads=4)
    b = shard_bounds(desc, 3)
    parts = []
    for r in range(3):
        local, sub, idx = slice_shard(batch, desc, int(b[r]), int(b[r + 1]))
        res, vst, _, _ = coracle.validate_proposals(local, sub, w.now, threads=2)
        parts.append(res)
        assert np.array_equal(vst, vst_ref[idx])
    assert np.concatenate(parts).tobytes() == ref.tobytes()


def _worker(rank, world, port, payload, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(os.path.dirname(here), "hashgraph-like-consensus_amd", "python"),
              os.path.join(os.path.dirname(here), "oracle"), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from hashgraph_like_consensus.batch import VoteBatch
    from hashgraph_like_consensus.parallel import validate_sharded
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        batch = VoteBatch(*payload["batch"])
        res, st = validate_sharded(OracleEngine(), batch, payload["desc"], payload["now"], want_votes=True)
        q.put((rank, res.tobytes(), st.tobytes()))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_sharded_equals_single():
    w = oracle_workload(5, 7, 9, False, seed=42)
    batch, desc, _ = byzantine(w, fraction=0.25, seed=9)
    ref, vst_ref, _, _ = coracle.validate_proposals(batch, desc, w.now, threads=4)
    payload = {"batch": (batch.vote_id, batch.proposal_id, batch.timestamp, batch.vote, batch.arena,
                         batch.field_off, batch.field_len), "desc": desc, "now": w.now}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, payload, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res, st in got:
        assert res == ref.tobytes(), f"rank {rank} results differ"
        assert st == vst_ref.tobytes(), f"rank {rank} vote statuses differ"


# ---- wire and streaming paths across ranks (gloo, world size 2) ----------------------------------
def _worker2(rank, world, port, kind, payload, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(os.path.dirname(here), "hashgraph-like-consensus_amd", "python"),
              os.path.join(os.path.dirname(here), "oracle"), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from oracle_engines import OracleEngine as OE
    from hashgraph_like_consensus.batch import VoteBatch
    from hashgraph_like_consensus.parallel import process_votes_sharded, validate_wire_sharded
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if kind == "wire":
            res, winfo = validate_wire_sharded(OE(), *payload)
            q.put((rank, res.tobytes() + winfo.tobytes()))
        else:
            batch = VoteBatch(*payload[0])
            out = process_votes_sharded(OE(), batch, *payload[1:])
            q.put((rank, b"".join(np.ascontiguousarray(o).tobytes() for o in out)))
    finally:
        dist.destroy_process_group()


def _run2(kind, payload):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker2, args=(r, 2, port, kind, payload, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def test_gloo_world2_wire_sharded_equals_single():
    import random
    from oracle_engines import OracleEngine as OE
    from hashgraph_like_consensus import _ffi, synth
    from hashgraph_like_consensus.protos import encode_proposal
    from wire_fuzz import mutate, random_proposal
    w = oracle_workload(5, 6, 8, True, seed=43)
    batch, desc, _ = byzantine(w, fraction=0.25, seed=11)
    wire, off, lens, scope = synth.to_wire(batch, desc)
    rnd = random.Random(3)
    extra = [mutate(rnd, encode_proposal(random_proposal(rnd, max_votes=2))) for _ in range(6)]
    ew = b"".join(extra)
    eo = np.cumsum([0] + [len(e) for e in extra[:-1]]).astype(np.uint64) + np.uint64(wire.size)
    wire = np.concatenate([wire, np.frombuffer(ew, np.uint8)])
    off = np.concatenate([off, eo])
    lens = np.concatenate([lens, np.array([len(e) for e in extra], np.uint32)])
    scope = np.concatenate([scope, scope[:1].repeat(len(extra))])
    ref_res, ref_w, _ = OE().validate_wire_proposals(wire, off, lens, scope, w.now)
    ref = ref_res.tobytes() + ref_w.tobytes()
    for rank, got in _run2("wire", (wire, off, lens, scope, w.now)):
        assert got == ref, f"rank {rank}: sharded wire outcomes differ"


def test_gloo_world2_stream_sharded_equals_single():
    from oracle_engines import OracleEngine as OE
    from stream_cases import device_inputs, streaming_workload
    sessions, votes, vs, now = streaming_workload(0x484C4340, n_props=8, votes=6)
    batch, vsess, sarr, owners, osess = device_inputs(sessions, votes, vs)
    ref_s = sarr.copy()
    st, tr, ins, rs = OE().process_votes(batch, vsess, ref_s, owners, osess, now)
    ref = b"".join(np.ascontiguousarray(o).tobytes() for o in (st, tr, ins, rs, ref_s))
    payload = ((batch.vote_id, batch.proposal_id, batch.timestamp, batch.vote, batch.arena, batch.field_off,
                batch.field_len), vsess, sarr, owners, osess, now)
    for rank, got in _run2("stream", payload):
        assert got == ref, f"rank {rank}: sharded streaming outcomes differ"


# ---- per-rank shards: each rank generates only its own proposals (config 4 style) -----------------
def _shard_workload(rank: int):
    from adversarial import byzantine
    w = oracle_workload(4, 6, 8, True, seed=0x484C4304, start=4 * rank)
    batch, desc, _ = byzantine(w, fraction=0.3, seed=100 + rank)
    return batch, desc, w.now


def _worker_shard(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(os.path.dirname(here), "hashgraph-like-consensus_amd", "python"),
              os.path.join(os.path.dirname(here), "oracle"), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from hashgraph_like_consensus.parallel import validate_shard
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        batch, desc, now = _shard_workload(rank)   # this rank's shard only
        if rank == 1:                               # ragged shards: rank 1 holds one proposal fewer
            desc = desc[:3].copy()
        res, st, counters = validate_shard(OracleEngine(), batch, desc, now, want_votes=True)
        q.put((rank, res.tobytes(), st.tobytes(), counters))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_rank_shards_gather_and_counters():
    """validate_shard: ranks hold disjoint, self-generated shards (no rank sees the whole batch);
    everyone receives all results in rank order and the all-reduced verified / rejected counters."""
    refs, sts = [], []
    hist_v = np.zeros(32, np.int64)
    hist_p = np.zeros(32, np.int64)
    for r in range(2):
        batch, desc, now = _shard_workload(r)
        if r == 1:
            desc = desc[:3].copy()
        res, vst, _, _ = coracle.validate_proposals(batch, desc, now, threads=2)
        idx = np.concatenate([np.arange(int(d["vote_begin"]), int(d["vote_begin"]) + int(d["vote_count"]))
                              for d in desc])
        refs.append(res.tobytes())
        sts.append(vst[idx].tobytes())
        hist_v += np.bincount(vst[idx], minlength=32)[:32]
        hist_p += np.bincount(res["status"], minlength=32)[:32]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_shard, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res, st, counters in got:
        assert res == b"".join(refs), f"rank {rank}: gathered results differ"
        assert st == b"".join(sts), f"rank {rank}: gathered statuses differ"
        assert counters["verified_votes"] == int(hist_v[0])
        assert counters["rejected_votes_by_status"] == {str(k): int(hist_v[k]) for k in range(1, 32) if hist_v[k]}
        assert counters["proposals_ok"] == int(hist_p[0])
        assert sum(counters["rejected_votes_by_status"].values()) > 0


# ---- config 4's true shard counts over 8 ranks ------------------------------------
C4_PROPOSALS, C4_RANKS, C4_V = 1_562_500, 8, 64


def _c4_span(rank: int):
    per = -(-C4_PROPOSALS // C4_RANKS)
    start = min(rank * per, C4_PROPOSALS)
    return start, min(per, C4_PROPOSALS - start)


def _c4_outputs(rank: int):
    """A deterministic stand-in for rank `rank`'s validated shard: 16-byte result rows (status, bad
    index, yes, total keyed to the global proposal index) and per-vote statuses with a sprinkling of
    reject codes -- what the exchange step moves, at the true config-4 proposal counts."""
    from hashgraph_like_consensus import _ffi
    start, P = _c4_span(rank)
    g = np.arange(start, start + P, dtype=np.int64)
    res = np.zeros(P, _ffi.RESULT_DTYPE)
    res["status"] = np.where(g % 97 == 0, 6, np.where(g % 89 == 0, 13, 0)).astype(np.uint8)
    res["transition"] = (g % 3).astype(np.uint8) * (res["status"] == 0)
    res["bad_index"] = np.where(res["status"] != 0, g % 64, 0xFFFFFFFF).astype(np.uint32)
    res["yes"] = (g * 7 % 65).astype(np.uint32)
    res["total"] = C4_V
    st = np.zeros(P * C4_V, np.uint8)
    bad = np.nonzero(res["status"] == 6)[0]
    st[bad * C4_V + (g[bad] % 64)] = 6
    return res, st


def _worker_c4(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(os.path.dirname(here), "hashgraph-like-consensus_amd", "python"), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from hashgraph_like_consensus.parallel import ShardExchange
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res, st = _c4_outputs(rank)
        P = res.shape[0]
        max_p = max(_c4_span(r)[1] for r in range(world))
        ex = ShardExchange(max_p, world, "cpu")
        ex(torch.from_numpy(res.view(np.uint8).copy()), torch.from_numpy(st), P, st.shape[0])
        pc = torch.tensor([P], dtype=torch.int64)
        pcs = [torch.zeros_like(pc) for _ in range(world)]
        dist.all_gather(pcs, pc)
        counts = [int(x.item()) for x in pcs]
        rows = ex.results(counts)
        q.put((rank, counts, rows.tobytes() == b"".join(_c4_outputs(r)[0].tobytes() for r in range(world)),
               ex.summary()))
    finally:
        dist.destroy_process_group()


def test_gloo_world8_config4_counts_gather_and_counters():
    """The exchange step of an 8-GPU config-4 run at its true shard sizes (7 x 195,313 + 195,309
    proposals, 12.5M per-vote statuses per rank), over gloo: every rank receives all 1,562,500 result
    rows in rank order, byte for byte, and the all-reduced counters equal the union's histograms."""
    hist_v = np.zeros(32, np.int64)
    hist_p = np.zeros(32, np.int64)
    for r in range(C4_RANKS):
        res, st = _c4_outputs(r)
        hist_v += np.bincount(st, minlength=32)[:32]
        hist_p += np.bincount(res["status"], minlength=32)[:32]
    assert int(hist_v.sum()) == C4_PROPOSALS * C4_V
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_c4, args=(r, C4_RANKS, port, q)) for r in range(C4_RANKS)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(g[0] for g in got) == list(range(C4_RANKS))
    for rank, counts, rows_ok, summary in got:
        assert counts == [195_313] * 7 + [195_309] and sum(counts) == C4_PROPOSALS
        assert rows_ok, f"rank {rank}: gathered rows differ"
        assert summary["verified_votes"] == int(hist_v[0])
        assert summary["rejected_votes_by_status"] == {str(k): int(hist_v[k]) for k in range(1, 32) if hist_v[k]}
        assert summary["proposals_ok"] == int(hist_p[0])
        assert summary["proposals_by_status"] == {str(k): int(hist_p[k]) for k in range(1, 32) if hist_p[k]}
