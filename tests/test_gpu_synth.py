"""Device-side workload generator (hlc_synth_votes_device) and BASELINE.json config 4.

* The GPU generator reproduces the Python generator (synth.py, signed by the C oracle) byte for
  byte: ids, timestamps, choices, arena (owners, chained vote hashes, RFC 6979 signatures),
  offsets, proposal records -- including non-zero shard starts and the j // 1024 timestamp step.
* Config 4 (100,000,000 votes = 1,562,500 proposals x 64 sharded by proposal over
  8 GPUs): each of the 8 rank shards (195,313 proposals, 12.5M votes; the last 195,309) generated on
  the device and validated through hlc_validate_proposals_device, one after another on this GPU -- all
  100M votes; full-size tally and counter properties per shard; a seeded 0.1 % sample of whole proposals is
  copied back and checked bit for bit against the C oracle, and three sampled proposals against
  the Python generator.  Proposals are independent (/root/reference/src/service.rs:263-279), so a
  shard is the whole job of its rank.
"""
import os

import numpy as np
import pytest

import coracle
from hashgraph_like_consensus import synth
from hashgraph_like_consensus.device import DeviceBatch
from helpers import oracle_workload

pytestmark = pytest.mark.gpu
THREADS = max(1, min(16, os.cpu_count() or 1))
CONFIG4_PROPOSALS = 1_562_500
CONFIG4_RANKS = 8


def _shard(rank: int, world: int = CONFIG4_RANKS, total: int = CONFIG4_PROPOSALS):
    per = -(-total // world)
    start = min(rank * per, total)
    return start, min(per, total - start)


def _same_as_python(db, w):
    b, d, priv = db.to_host()
    for f in ("vote_id", "proposal_id", "timestamp", "vote", "arena", "field_off", "field_len"):
        assert np.array_equal(getattr(b, f), getattr(w.batch, f)), f
    assert d.tobytes() == w.desc.tobytes()
    if priv is not None:
        assert np.array_equal(priv, w.priv)


@pytest.mark.parametrize("P,V,expected,gossip,start", [(3, 5, 5, True, 0), (4, 64, 64, True, 1234),
                                                       (1, 1100, 1500, False, 7), (2, 1, 3, True, 0)])
def test_gpu_synth_equals_python_generator(engine, P, V, expected, gossip, start):
    seed = synth.config_seed(4) + P
    db = DeviceBatch.synthetic(engine, P, V, expected, gossip, seed, start_proposal=start, want_priv=True)
    w = oracle_workload(P, V, expected, gossip, seed, start=start)
    _same_as_python(db, w)


def test_gpu_synth_shard_starts():
    """The rank shards of config 4 tile the 1,562,500 proposals exactly."""
    spans = [_shard(r) for r in range(CONFIG4_RANKS)]
    assert spans[0] == (0, 195_313) and spans[-1] == (1_367_191, 195_309)
    assert sum(c for _, c in spans) == CONFIG4_PROPOSALS
    assert all(spans[r][0] + spans[r][1] == spans[r + 1][0] for r in range(CONFIG4_RANKS - 1))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("rank", list(range(CONFIG4_RANKS)))
def test_gpu_config4_rank_shard(engine, rank):
    """Every rank shard of config 4 in turn: all 100,000,000 votes through the HIP path.  Full-size
    properties per shard (every vote valid, every proposal Ok with its 64 votes, each proposal's YES tally
    equal to its votes' choices, each transition the reference's tally of that count, the outcome
    counters of the exchange step equal to the statuses), plus the 0.1 % oracle sample."""
    import torch
    start, P = _shard(rank)
    V = 64
    seed = synth.config_seed(4)
    db = DeviceBatch.synthetic(engine, P, V, V, True, seed, start_proposal=start)
    db.want_recovered()
    engine.validate_proposals_device(db)
    torch.cuda.synchronize()
    res = db.results_numpy()
    st = db.status_numpy()
    assert db.n == P * V
    assert (st == 0).all(), f"{int((st != 0).sum())} valid votes rejected"
    assert (res["status"] == 0).all() and (res["total"] == V).all()
    # full-size tally properties: YES = the proposal's choices; transition = calculate_consensus_result
    yes = db.choice_numpy().reshape(P, V).astype(np.int64).sum(axis=1)
    assert np.array_equal(res["yes"].astype(np.int64), yes)
    want = {}
    for y in np.unique(yes):
        r = coracle.consensus_result(V, int(y), V, 2.0 / 3.0, True, False)
        want[int(y)] = 0 if r is None else (2 if r else 1)
    assert np.array_equal(res["transition"], np.vectorize(want.get)(yes).astype(np.uint8))
    # the exchange step's outcome counters (hlc_outcome_counts_device) on the whole shard
    counts = torch.zeros(64, dtype=torch.int64, device=db.device)
    engine.outcome_counts_device(db.status.data_ptr(), db.n, db.results.data_ptr(), P, counts.data_ptr())
    torch.cuda.synchronize()
    c = counts.cpu().numpy()
    assert c[0] == db.n and c[1:32].sum() == 0 and c[32] == P and c[33:].sum() == 0
    # 0.1 % seeded sample of whole proposals, bit for bit against the C oracle
    rng = np.random.default_rng(0x484C4304 + rank)
    pick = np.sort(rng.choice(P, size=max(1, P // 1000), replace=False))
    hb, hd, vidx = db.host_proposals(pick)
    cres, cvst, cvrs, crec = coracle.validate_proposals(hb, hd, db.now, threads=THREADS)
    tv = torch.from_numpy(vidx).to(db.device)
    gst = db.status.index_select(0, tv).cpu().numpy()
    grs = db.reason.index_select(0, tv).cpu().numpy()
    grec = db.recovered[: db.n * 20].view(-1, 20).index_select(0, tv).cpu().numpy()
    assert np.array_equal(gst, cvst) and np.array_equal(grs, cvrs)
    assert np.array_equal(grec, crec)
    assert res[pick].tobytes() == cres.tobytes()
    # the device generator equals the Python one at these global proposal indices
    for k in pick[:3]:
        w = oracle_workload(1, V, V, True, seed, start=start + int(k))
        b1, d1, _ = db.host_proposals([int(k)])
        assert np.array_equal(b1.vote_id, w.batch.vote_id) and np.array_equal(b1.vote, w.batch.vote)
        for i in range(V):
            for f in range(5):
                assert b1.field(i, f) == w.batch.field(i, f)
        d1["vote_begin"] = 0
        assert d1.tobytes() == w.desc.tobytes()
