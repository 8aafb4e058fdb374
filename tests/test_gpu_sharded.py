"""The sharded entry paths (parallel.py) with the real HIP engine: two processes on the one GPU of
the box (gloo for the result exchange), each validating its shard through libhlc.so; the
gathered outcomes must equal one whole-batch call -- proposal-, wire- and session-sharded."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs():
    from adversarial import byzantine
    from hashgraph_like_consensus import synth
    from helpers import oracle_workload
    from stream_cases import device_inputs, streaming_workload
    w = oracle_workload(12, 10, 10, True, seed=0x484C4350)
    batch, desc, _ = byzantine(w, fraction=0.2, seed=12)
    wire, off, lens, scope = synth.to_wire(batch, desc)
    sessions, votes, vs, now = streaming_workload(0x484C4351, n_props=10, votes=8)
    sb, vsess, sarr, owners, osess = device_inputs(sessions, votes, vs)
    return (batch, desc, w.now), (wire, off, lens, scope, w.now), (sb, vsess, sarr, owners, osess, now)


def _flat(batch):
    return (batch.vote_id, batch.proposal_id, batch.timestamp, batch.vote, batch.arena, batch.field_off,
            batch.field_len)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(os.path.dirname(here), "hashgraph-like-consensus_amd", "python"),
              os.path.join(os.path.dirname(here), "oracle"), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from hashgraph_like_consensus.engine import Engine
    from hashgraph_like_consensus.parallel import process_votes_sharded, validate_sharded, validate_wire_sharded
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = Engine(0)
    try:
        (batch, desc, now), wire_in, (sb, vsess, sarr, owners, osess, snow) = _inputs()
        r1, _ = validate_sharded(eng, batch, desc, now, device="cpu")
        r2, w2 = validate_wire_sharded(eng, *wire_in, device="cpu")
        st, tr, ins, rs, fin = process_votes_sharded(eng, sb, vsess, sarr, owners, osess, snow, device="cpu")
        q.put((rank, [r1.tobytes(), r2.tobytes(), w2.tobytes(), st.tobytes(), tr.tobytes(), ins.tobytes(),
                      rs.tobytes(), fin.tobytes()]))
    finally:
        eng.close()
        dist.destroy_process_group()


def test_gpu_sharded_paths_equal_single(engine):
    (batch, desc, now), (wire, off, lens, scope, wnow), (sb, vsess, sarr, owners, osess, snow) = _inputs()
    r1, _, _, _ = engine.validate_proposals(batch, desc, now, want_votes=False)
    r2, w2, _ = engine.validate_wire_proposals(wire, off, lens, scope, wnow)
    fin = sarr.copy()
    st, tr, ins, rs = engine.process_votes(sb, vsess, fin, owners, osess, snow)
    ref = [r1.tobytes(), r2.tobytes(), w2.tobytes(), st.tobytes(), tr.tobytes(), ins.tobytes(), rs.tobytes(),
           fin.tobytes()]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=200) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    names = ["proposal results", "wire results", "wire info", "stream status", "stream transition",
             "stream inserted", "stream reason", "final sessions"]
    for rank, parts in got:
        for name, a, b in zip(names, parts, ref):
            assert a == b, f"rank {rank}: sharded {name} differ from the single call"


def _rccl_worker(port, q):
    """One rank over RCCL (world size 1): the exchange bench.py's N > 1 step runs on device tensors
    (ShardExchange: all_gather_into_tensor of the result rows, all_reduce of the counters) and the
    proposal-sharded entry (validate_shard), on the GPU."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(os.path.dirname(here), "hashgraph-like-consensus_amd", "python"),
              os.path.join(os.path.dirname(here), "oracle"), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from hashgraph_like_consensus.device import DeviceBatch
    from hashgraph_like_consensus.engine import Engine
    from hashgraph_like_consensus.parallel import ShardExchange, validate_shard
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    eng = Engine(0)
    try:
        db = DeviceBatch.synthetic(eng, 300, 64, 64, True, 0x484C4352, device="cuda:0")
        stream = torch.cuda.Stream(device="cuda:0")
        ex = ShardExchange(300, 1, "cuda:0", engine=eng)
        eng.validate_proposals_device(db, stream.cuda_stream)
        with torch.cuda.stream(stream):
            ex(db.results, db.status, 300, db.n)
        torch.cuda.synchronize()
        rows = ex.results([300])
        same = rows.view(np.uint8).tobytes() == db.results_numpy().view(np.uint8).tobytes()
        summ = ex.summary()
        (batch, desc, now), _, _ = _inputs()
        full, vst, summ2 = validate_shard(eng, batch, desc, now, device="cuda:0", want_votes=True)
        q.put((same, summ, db.n, full.tobytes(), vst.tobytes(), summ2))
    finally:
        eng.close()
        dist.destroy_process_group()


def test_gpu_rccl_exchange_one_rank(engine):
    """The RCCL branch of the exchange (the driver's multi-GPU bench runs it at N = 2, 4, 8) at one
    rank on the box's GPU: gathered rows equal the local results, counters count every vote, and the
    proposal-sharded entry over RCCL equals the single call."""
    (batch, desc, now), _, _ = _inputs()
    res, vst, _, _ = engine.validate_proposals(batch, desc, now, want_votes=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    same, summ, n, full, vrows, summ2 = q.get(timeout=200)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert same, "RCCL-gathered rows differ from the local results"
    assert summ["verified_votes"] == n and summ["proposals_ok"] == 300
    assert full == res.tobytes()
    idx = np.concatenate([np.arange(int(d["vote_begin"]), int(d["vote_begin"]) + int(d["vote_count"]))
                          for d in desc])
    assert vrows == np.asarray(vst, np.uint8)[idx].tobytes()
    assert summ2["verified_votes"] == int((np.asarray(vst)[idx] == 0).sum())
