"""Config-2 throughput with batches overlapping on the device (GPU box): K calls of
hlc_validate_proposals_device over the same 640k-vote batch, issued round-robin over `--inflight`
contexts, each on its own stream with its own output buffers, so call k+1's prep / main stages can
fill call k's grid tail and its comb / final / tally.  Outputs of every context are checked equal
to the one-context run before timing.

    python tools/inflight.py --steps 150 --warmup 50 --inflight 1,2,3
"""
from __future__ import annotations

import argparse
import copy
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hashgraph-like-consensus_amd", "python"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--inflight", default="1,2")
    ap.add_argument("--proposals", type=int, default=10_000, help="64 votes each (2048 = one 131k-vote pipeline chunk)")
    a = ap.parse_args()
    import numpy as np
    import torch

    from hashgraph_like_consensus import _ffi, synth
    from hashgraph_like_consensus.device import DeviceBatch
    from hashgraph_like_consensus.engine import Engine

    engines = [Engine(0)]
    db = DeviceBatch.synthetic(engines[0], a.proposals, 64, 64, True, synth.config_seed(2))
    torch.cuda.synchronize()

    def twin():
        t = copy.copy(db)
        t.results = torch.zeros_like(db.results)
        t.status = torch.zeros_like(db.status)
        t.reason = torch.zeros_like(db.reason)
        t.results_ptr = ctypes.cast(t.results.data_ptr(), ctypes.POINTER(_ffi.hlc_result))
        t.status_ptr = ctypes.cast(t.status.data_ptr(), ctypes.POINTER(ctypes.c_uint8))
        t.reason_ptr = ctypes.cast(t.reason.data_ptr(), ctypes.POINTER(ctypes.c_uint8))
        return t

    out = []
    for k in [int(x) for x in a.inflight.split(",")]:
        while len(engines) < k:
            engines.append(Engine(0))
        for e in engines[:k]:
            e.reserve(db.n, db.n_proposals, db.bytes_len)
        batches = [twin() for _ in range(k)]
        streams = [torch.cuda.Stream() for _ in range(k)]
        for i in range(a.warmup):
            j = i % k
            engines[j].validate_proposals_device(batches[j], streams[j].cuda_stream)
        torch.cuda.synchronize()
        for b in batches:
            assert (b.status_numpy() == 0).all() and (b.results_numpy()["status"] == 0).all()
        t0 = time.perf_counter()
        for i in range(a.steps):
            j = i % k
            engines[j].validate_proposals_device(batches[j], streams[j].cuda_stream)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        row = {"votes": db.n, "inflight": k, "steps": a.steps, "ms_per_step": el / a.steps * 1e3, "votes_per_s": db.n * a.steps / el}
        print(json.dumps(row), flush=True)
        out.append(row)
    for e in engines:
        e.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
