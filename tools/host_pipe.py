"""The host-buffer entry hlc_validate_proposals (what the Rust process_incoming_proposals of
INTEGRATION.md calls) on the config-2 workload (GPU box).

For each setting of the range schedule (hlc_api.cpp validate_host: HLC_SPLIT_VOTES, HLC_HOST_THREADS,
read on every call): outputs equal the first setting's bit for
bit, then --steps calls are timed (host buffers in, per-vote statuses + per-proposal results out,
blocking).

    python tools/host_pipe.py --steps 10 --split 0/131072/131072,196608 --threads 4,8 --rounds 2
    (HLC_HOST_TRACE=1 in the environment adds each call's timeline on stderr)
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
    """HLC_HOST_TRACE lines (hlc_api.cpp HostTrace): host phase ends | device event times, ms."""
    for line in open(path):
        if not line.startswith("HLC_HOST_TRACE "):
            continue
        d = json.loads(line[len("HLC_HOST_TRACE "):])
        print("host  " + "  ".join(f"{k} {v:.2f}" for k, v in d["host"].items()))
        print("  dev " + "  ".join(f"{k} {v:.2f}" for k, v in d["device"].items()))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--split", default="98304,196608", help="'/'-separated HLC_SPLIT_VOTES settings (range sizes "
                    "before the last, e.g. 131072,196608/0; 0 = one recovery range)")
    ap.add_argument("--threads", default="16", help="HLC_HOST_THREADS settings")
    ap.add_argument("--nt", default="1", help="','-separated HLC_NT_COPY settings (non-temporal staging copies)")
    ap.add_argument("--bind", default="1", help="','-separated HLC_POOL_BIND settings (staging workers on the GPU's "
                    "NUMA node)")
    ap.add_argument("--rounds", type=int, default=1, help="alternate the whole sweep this many times (box drift)")
    ap.add_argument("--proposals", type=int, default=10_000)
    ap.add_argument("--pinned", action="store_true", help="the host batch in page-locked memory (hlc_host_alloc)")
    ap.add_argument("--print-trace", default=None, help="print an HLC_HOST_TRACE log as a table and exit")
    ap.add_argument("--contexts", type=int, default=1,
                    help="also time this many contexts, one caller thread each, every thread calling back to back "
                         "(include/hlc.h: one context per thread for concurrency); aggregate votes/s")
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
    if a.pinned:
        b = b.pinned()
    torch.cuda.synchronize()
    bytes_in = int(b.arena.nbytes + b.vote_id.nbytes + b.proposal_id.nbytes + b.timestamp.nbytes + b.vote.nbytes
                   + b.field_off.nbytes + b.field_len.nbytes + d.nbytes)
    ref = None
    settings = [(sp, th, nt, bd) for sp in a.split.split("/") for th in a.threads.split(",")
                for nt in a.nt.split(",") for bd in a.bind.split(",")] * max(1, a.rounds)
    for sp, th, nt, bd in settings:
        eng.set_option("nt_copy", int(nt))  # hlc_ctx_set_option (the environment is read at creation only)
        eng.set_option("pool_bind", int(bd))
        eng.set_option("split_votes", sp)
        eng.set_option("host_threads", int(th))
        r = eng.validate_proposals(b, d, db.now, want_votes=True)
        if ref is None:
            ref = r
            assert (r[1] == 0).all() and (r[0]["status"] == 0).all()
        assert np.array_equal(r[0], ref[0]) and np.array_equal(r[1], ref[1]) and np.array_equal(r[2], ref[2])
        t = time.perf_counter()
        for _ in range(a.steps):
            eng.validate_proposals(b, d, db.now, want_votes=True)
        el = (time.perf_counter() - t) / a.steps
        row = {"split": sp, "threads": int(th), "nt_copy": int(nt), "pool_bind": int(bd), "pinned": a.pinned,
               "ms_per_call": el * 1e3,
               "votes_per_s": b.n / el, "bytes_in_per_call": bytes_in, "outputs_equal_first_setting": True}
        print(json.dumps(row), flush=True)
    if a.contexts > 1:
        import threading
        engs = [eng] + [Engine(0) for _ in range(a.contexts - 1)]
        for e in engs[1:]:
            for k in ("nt_copy", "pool_bind", "host_threads"):
                e.set_option(k, eng.get_option(k))
            e.set_option("split_votes", settings[-1][0])
            e.validate_proposals(b, d, db.now, want_votes=True)  # warm: workspace, staging, streams
        go = threading.Barrier(a.contexts + 1)
        times = [0.0] * a.contexts

        def work(k):
            go.wait()
            t = time.perf_counter()
            for _ in range(a.steps):
                engs[k].validate_proposals(b, d, db.now, want_votes=True)
            times[k] = time.perf_counter() - t

        th = [threading.Thread(target=work, args=(k,)) for k in range(a.contexts)]
        for x in th:
            x.start()
        go.wait()
        for x in th:
            x.join()
        el = max(times)
        print(json.dumps({"contexts": a.contexts, "threads_per_context": eng.get_option("host_threads"),
                          "split": settings[-1][0], "calls": a.contexts * a.steps,
                          "votes_per_s_aggregate": a.contexts * a.steps * b.n / el,
                          "ms_per_call_mean": el / a.steps * 1e3}), flush=True)
        for e in engs[1:]:
            e.close()
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
