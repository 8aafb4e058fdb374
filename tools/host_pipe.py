"""The host-buffer entry hlc_validate_proposals (what the Rust process_incoming_proposals of
INTEGRATION.md calls) on the config-2 workload, one-shot vs pipelined (GPU box).

The pipeline chunk size is read from HLC_PIPE_CHUNK_VOTES on every call (0 = one-shot).  For each
setting: outputs equal the one-shot outputs bit for bit, then --steps calls are timed (host buffers
in, per-vote statuses + per-proposal results out, blocking).

    python tools/host_pipe.py --steps 10 --chunks 0,65536,131072,262144 --depths 2,3,4
    (HLC_PIPE_TRACE=1 in the environment adds the per-chunk timeline of every call on stderr)
    python tools/host_pipe.py --print-trace gpurun_out/trace.txt   (that timeline as a table; no GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hashgraph-like-consensus_amd", "python"))


def print_trace(path: str) -> None:
    """HLC_PIPE_TRACE lines (hlc_api.cpp PipeTrace) as one row per chunk: host phases (wait for the
    child's inputs, staging end, enqueue ends) | device spans (H2D, kernels end, D2H end), ms."""
    for line in open(path):
        if not line.startswith("HLC_PIPE_TRACE "):
            continue
        d = json.loads(line[len("HLC_PIPE_TRACE "):])
        print(f"{d['votes']} votes, {d['chunks']} chunks, host {d['host_ms']:.2f} ms")
        for r in d["rows"]:
            print(f"  wait {r['wait'][0]:6.2f}-{r['wait'][1]:6.2f} stage {r['stage_end']:6.2f} "
                  f"enq {r.get('enq_h2d_end', -1):6.2f}/{r.get('enq_kern_end', -1):6.2f}/{r['enq_end']:6.2f} | "
                  f"h2d {r['h2d'][0]:6.2f}-{r['h2d'][1]:6.2f} kern_end {r['kern_end']:6.2f} d2h_end {r['d2h_end']:6.2f}")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--chunks", default="0,65536,131072,262144")
    ap.add_argument("--threads", default="4", help="HLC_PIPE_THREADS settings to sweep")
    ap.add_argument("--depths", default="3", help="HLC_PIPE_DEPTH settings to sweep (child contexts in flight)")
    ap.add_argument("--proposals", type=int, default=10_000)
    ap.add_argument("--schedules", default="", help="';'- or '/'-separated HLC_PIPE_CHUNKS schedules (votes of chunks 0, 1, "
                    "...; the last size repeats), each run at every depth / thread setting; replaces --chunks")
    ap.add_argument("--streams", default="own", help="HLC_PIPE_STREAMS settings to sweep (own, shared)")
    ap.add_argument("--rounds", type=int, default=1, help="alternate the whole sweep this many times (box drift)")
    ap.add_argument("--print-trace", default=None, help="print an HLC_PIPE_TRACE log as a table and exit")
    a = ap.parse_args()
    if a.print_trace:
        print_trace(a.print_trace)
        return 0
    import numpy as np
    import torch

    from hashgraph_like_consensus import synth
    from hashgraph_like_consensus.device import DeviceBatch
    from hashgraph_like_consensus.engine import Engine

    eng = Engine(0)
    db = DeviceBatch.synthetic(eng, a.proposals, 64, 64, True, synth.config_seed(2))
    b, d, _ = db.to_host()
    torch.cuda.synchronize()
    bytes_in = int(b.arena.nbytes + b.vote_id.nbytes + b.proposal_id.nbytes + b.timestamp.nbytes + b.vote.nbytes
                   + b.field_off.nbytes + b.field_len.nbytes + d.nbytes)
    ref = None
    out = []
    chunks = [("0", 0)] + [(x, 65536) for x in a.schedules.replace("/", ";").split(";") if x] if a.schedules else \
        [("", int(x)) for x in a.chunks.split(",")]
    settings = [(sc, c, t, dp, sm) for sc, c in chunks for t in [int(x) for x in a.threads.split(",")]
                for dp in [int(x) for x in a.depths.split(",")] for sm in a.streams.split(",")] * max(1, a.rounds)
    for sched, c, th, dp, sm in settings:
        os.environ["HLC_PIPE_STREAMS"] = sm
        if c == 0 and ref is not None:
            continue
        if sched and sched != "0":
            os.environ["HLC_PIPE_CHUNKS"] = sched
        else:
            os.environ.pop("HLC_PIPE_CHUNKS", None)
        os.environ["HLC_PIPE_CHUNK_VOTES"] = str(c)
        os.environ["HLC_PIPE_THREADS"] = str(th)
        os.environ["HLC_PIPE_DEPTH"] = str(dp)
        r = eng.validate_proposals(b, d, db.now, want_votes=True)
        if ref is None:
            ref = r
            assert (r[1] == 0).all() and (r[0]["status"] == 0).all()
        assert np.array_equal(r[0], ref[0]) and np.array_equal(r[1], ref[1]) and np.array_equal(r[2], ref[2])
        t = time.perf_counter()
        for _ in range(a.steps):
            eng.validate_proposals(b, d, db.now, want_votes=True)
        el = (time.perf_counter() - t) / a.steps
        row = {"chunk_votes": c, "schedule": sched, "threads": th, "depth": dp, "streams": sm, "ms_per_call": el * 1e3, "votes_per_s": b.n / el, "bytes_in_per_call": bytes_in,
               "outputs_equal_one_shot": True}
        print(json.dumps(row), flush=True)
        out.append(row)
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
