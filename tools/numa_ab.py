"""A/B of the host-buffer entry's staging placement when the caller's inputs sit on the far NUMA node
(the driver's round-5 run had its pageable inputs on node 1, the GPU on node 0).

The config-2 batch (640k votes, generated on the GPU) is copied into fresh arrays by this thread while
it is pinned to the CPUs of one NUMA node -- the first touch puts the pages there -- once on a node
other than the GPU's ("far") and once on the GPU's ("near").  Then hlc_validate_proposals runs on each
copy with the staging workers bound by HLC_OPT_POOL_BIND = 1 (the GPU's node, the round-5 default),
2 (the node the call's arena lives on) and 0 (unbound), the arms interleaved over `--rounds`; each row
carries the traced phase ends (rest_staged / rest_landed) of one extra call.  The page-locked leg
(hlc_host_alloc inputs, no staging) is the ceiling.  Every call's outputs equal the first call's.

  python tools/numa_ab.py --steps 10 --rounds 3 > gpurun_out/numa_ab.txt
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hashgraph-like-consensus_amd", "python"))
sys.path.insert(0, ROOT)


def node_cpus():
    import bench
    base = "/sys/devices/system/node"
    aff = os.sched_getaffinity(0)
    out = {}
    for d in sorted(os.listdir(base)):
        if d.startswith("node") and d[4:].isdigit():
            with open(f"{base}/{d}/cpulist") as f:
                cpus = bench._cpulist(f.read()) & aff
            if cpus:
                out[int(d[4:])] = cpus
    return out


def copy_on(batch, cpus):
    """A copy of every array of `batch` first-touched by this thread pinned to `cpus`."""
    import numpy as np

    from hashgraph_like_consensus.batch import VoteBatch
    old = os.sched_getaffinity(0)
    os.sched_setaffinity(0, cpus)
    try:
        def fresh(a):
            out = np.empty_like(a)
            out[...] = a  # the first write to each page happens here, on `cpus`
            return out
        return VoteBatch(*(fresh(getattr(batch, f)) for f in ("vote_id", "proposal_id", "timestamp", "vote", "arena",
                                                             "field_off", "field_len")))
    finally:
        os.sched_setaffinity(0, old)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--proposals", type=int, default=10_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--binds", default="1,2,0")
    a = ap.parse_args()

    import numpy as np
    import torch

    import bench
    from hashgraph_like_consensus import synth
    from hashgraph_like_consensus.device import DeviceBatch
    from hashgraph_like_consensus.engine import Engine

    eng = Engine(0)
    db = DeviceBatch.synthetic(eng, a.proposals, 64, 64, True, synth.config_seed(2))
    b, d, _ = db.to_host()
    torch.cuda.synchronize()
    facts = bench.numa_facts(torch, "cuda:0", [b.arena])
    gpu_node = facts.get("gpu_numa_node")
    nodes = node_cpus()
    print(json.dumps({"gpu_numa_node": gpu_node, "nodes_cpus": {k: len(v) for k, v in nodes.items()},
                      "host_threads": eng.get_option("host_threads")}), flush=True)
    far_nodes = [k for k in nodes if k != gpu_node]
    copies = {}
    if far_nodes:
        copies["far"] = copy_on(b, nodes[far_nodes[0]])
    if gpu_node in nodes:
        copies["near"] = copy_on(b, nodes[gpu_node])
    for name, cb in copies.items():
        f = bench.numa_facts(torch, "cuda:0", [cb.arena, cb.field_off])
        print(json.dumps({"inputs": name, "input_pages_by_node": f.get("input_pages_by_node")}), flush=True)
    ref = eng.validate_proposals(b, d, db.now, want_votes=True)
    assert (ref[1] == 0).all() and (ref[0]["status"] == 0).all()
    rows = {}
    for rnd in range(a.rounds):
        for name, cb in copies.items():
            for bind in (int(x) for x in a.binds.split(",")):
                eng.set_option("pool_bind", bind)
                r = eng.validate_proposals(cb, d, db.now, want_votes=True)
                assert all(np.array_equal(x, y) for x, y in zip(r[:3], ref[:3])), (name, bind)
                t = time.perf_counter()
                for _ in range(a.steps):
                    eng.validate_proposals(cb, d, db.now, want_votes=True)
                el = (time.perf_counter() - t) / a.steps
                with eng.options(host_trace=2):
                    eng.validate_proposals(cb, d, db.now, want_votes=True)
                    tr = eng.last_host_trace()
                row = {"round": rnd, "inputs": name, "pool_bind": bind, "ms_per_call": el * 1e3,
                       "votes_per_s": b.n / el, "rest_staged_ms": tr["host"].get("rest_staged"),
                       "rest_landed_ms": tr["device"].get("rest_landed"),
                       "outputs_landed_ms": tr["device"].get("outputs_landed"),
                       **{k: tr.get("facts", {}).get(k) for k in ("pool_cpus", "pool_node", "arena_node", "staging_node",
                                                                  "gpu_node")}}
                rows.setdefault((name, bind), []).append(row["votes_per_s"])
                print(json.dumps(row), flush=True)
    eng.set_option("pool_bind", 1)
    pb = b.pinned()
    eng.validate_proposals(pb, d, db.now, want_votes=True)
    t = time.perf_counter()
    for _ in range(a.steps):
        eng.validate_proposals(pb, d, db.now, want_votes=True)
    el = (time.perf_counter() - t) / a.steps
    summary = {f"{k[0]}/bind{k[1]}": statistics.median(v) for k, v in rows.items()}
    summary["page_locked"] = b.n / el
    print(json.dumps({"median_votes_per_s": summary}), flush=True)
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
