#!/usr/bin/env python3
"""Regenerates the golden fixtures in tests/golden/*.npz (inputs + expected outputs).

Inputs are deterministic (fixed keys, seeded RNG, RFC 6979 signatures).  Expected outputs come
from the C restatement and are asserted equal to the Python restatement before being written, so
a fixture is only produced when the two independent oracles agree.  Run from the repo root:
    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "hashgraph-like-consensus_amd", "python"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import coracle  # noqa: E402
import pyoracle as po  # noqa: E402
from adversarial import byzantine, config_of, proposals_from_batch  # noqa: E402
from hashgraph_like_consensus.batch import ProposalConfig, pack_proposals  # noqa: E402
from helpers import oracle_workload  # noqa: E402
from scenarios import scenarios  # noqa: E402


def save(name, batch, desc, now):
    res, vst, vrs, rec = coracle.validate_proposals(batch, desc, now, threads=4)
    props = proposals_from_batch(batch, desc)
    b = 0
    for k, p in enumerate(props):
        out = po.from_proposal(p, config_of(desc[k]), now)
        assert int(res[k]["status"]) == out.status, (name, k)
        assert int(res[k]["transition"]) == out.transition, (name, k)
        for j, v in enumerate(p.votes):
            assert (int(vst[b + j]), int(vrs[b + j])) == po.vote_status_in_proposal(p, v, now), (name, k, j)
        b += len(p.votes)
    np.savez_compressed(
        os.path.join(HERE, name + ".npz"), vote_id=batch.vote_id, proposal_id=batch.proposal_id,
        timestamp=batch.timestamp, vote=batch.vote, arena=batch.arena, field_off=batch.field_off,
        field_len=batch.field_len, desc=desc.view(np.uint8).reshape(len(desc), -1), now=np.uint64(now),
        exp_results=res.view(np.uint8).reshape(len(res), -1), exp_vote_status=vst, exp_vote_reason=vrs,
        exp_recovered=rec)
    print(name, batch.n, "votes", len(desc), "proposals", sorted(set(int(x) for x in res["status"])))


def main():
    # BASELINE config 1: Gossipsub, 1 proposal, 3 voters (rfc_compliance_tests.rs:423-488 shape)
    w = oracle_workload(1, 3, 3, True, 0x484C4301, name="config1")
    save("config1_gossipsub_3_voters", w.batch, w.desc, w.now)
    # the reference's behavioural tests, one fixture per `now`
    sc = scenarios()
    for t, now in enumerate(sorted({s[3] for s in sc})):
        items = [s for s in sc if s[3] == now]
        batch, desc = pack_proposals([p for _, p, _, _, _ in items],
                                     [ProposalConfig(c.consensus_threshold, c.max_rounds, c.use_gossipsub_rounds)
                                      for _, _, c, _, _ in items])
        save(f"scenarios_{t}", batch, desc, now)
    # config 5 shape, small: 1/3 Byzantine votes over every mutation kind
    w = oracle_workload(12, 16, 16, True, 0x484C4305)
    batch, desc, _ = byzantine(w, fraction=1 / 3, seed=5)
    save("config5_byzantine_small", batch, desc, w.now)


if __name__ == "__main__":
    main()
