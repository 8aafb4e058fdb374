"""The wire entry from host buffers, hlc_validate_wire_proposals (gossip bytes of consensus.proto
Proposal messages in host memory -> per-proposal results), on the config-2 workload (GPU box).

For each setting of the pipelined schedule (hlc_api.cpp validate_wire_host: HLC_WIRE_SPLIT_BYTES,
HLC_WIRE_CHUNK, HLC_HOST_THREADS, read on every call; "plain" = HLC_WIRE_PIPELINE=0, the unpipelined
arm): outputs equal the device-resident SoA path's bit for bit, then --steps calls are timed.

    python tools/wire_pipe.py --steps 10 --split default/16777216,33554432/plain --chunk 4194304,8388608
    (HLC_HOST_TRACE=1 adds each call's timeline on stderr; --trace prints one traced call per setting)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hashgraph-like-consensus_amd", "python"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--split", default="default",
                    help="'/'-separated HLC_WIRE_SPLIT_BYTES settings ('plain' = the unpipelined arm, 'default' = "
                    "the library's schedule)")
    ap.add_argument("--chunk", default="4194304", help="','-separated HLC_WIRE_CHUNK settings (the library default: 4 MiB)")
    ap.add_argument("--threads", default="16", help="','-separated HLC_HOST_THREADS settings")
    ap.add_argument("--nt", default="1", help="','-separated HLC_NT_COPY settings (non-temporal staging copies)")
    ap.add_argument("--bind", default="1", help="','-separated HLC_POOL_BIND settings (staging workers on the GPU's "
                    "NUMA node)")
    ap.add_argument("--walk", default="", help="','-separated HLC_WIRE_WALK settings for the pipelined entry "
                    "(lane / lds; empty = the library default)")
    ap.add_argument("--rounds", type=int, default=1, help="alternate the whole sweep this many times (box drift)")
    ap.add_argument("--proposals", type=int, default=10_000)
    ap.add_argument("--pinned", action="store_true", help="the wire bytes in page-locked memory (hlc_host_alloc)")
    ap.add_argument("--trace", action="store_true", help="one extra traced call per setting (HLC_HOST_TRACE=2)")
    ap.add_argument("--device-walk", default="", help="also time the device-resident wire entry "
                    "(hlc_validate_wire_proposals_device) under these ','-separated HLC_WIRE_WALK settings")
    a = ap.parse_args()
    import numpy as np
    import torch

    from hashgraph_like_consensus import _ffi, synth
    from hashgraph_like_consensus.device import DeviceBatch
    from hashgraph_like_consensus.engine import Engine

    eng = Engine(0)
    db = DeviceBatch.synthetic(eng, a.proposals, 64, 64, True, synth.config_seed(2))
    eng.validate_proposals_device(db)
    torch.cuda.synchronize()
    ref = db.results_numpy()
    b, d, _ = db.to_host()
    wire, off, lens, scope = synth.to_wire(b, d)
    arena = None
    if a.pinned:
        arena = _ffi.PinnedArena(wire.size + 64)
        pw = arena.take(wire.shape, np.uint8)
        pw[:] = wire
        wire = pw
    settings = [(sp, ch, th, nt, bd, wk) for sp in a.split.split("/") for ch in a.chunk.split(",")
                for th in a.threads.split(",") for nt in a.nt.split(",") for bd in a.bind.split(",")
                for wk in a.walk.split(",")] * max(1, a.rounds)
    for sp, ch, th, nt, bd, wk in settings:
        # hlc_ctx_set_option (the environment is read at context creation only)
        eng.set_option("wire_walk", {"lane": 0, "lds": 1}.get(wk, -1))
        eng.set_option("nt_copy", int(nt))
        eng.set_option("pool_bind", int(bd))
        eng.set_option("wire_pipeline", 0 if sp == "plain" else 1)
        if sp == "default":
            eng.set_option("wire_split_bytes", -1)
        elif sp != "plain":
            eng.set_option("wire_split_bytes", sp)
        eng.set_option("wire_chunk", int(ch))
        eng.set_option("host_threads", int(th))
        res, winfo, nv = eng.validate_wire_proposals(wire, off, lens, scope, db.now)
        assert np.array_equal(res, ref) and nv == db.n and (winfo["decode_status"] == 0).all(), sp
        t = time.perf_counter()
        for _ in range(a.steps):
            eng.validate_wire_proposals(wire, off, lens, scope, db.now)
        el = (time.perf_counter() - t) / a.steps
        row = {"split": sp, "chunk": int(ch), "threads": int(th), "nt_copy": int(nt), "pool_bind": int(bd),
               "walk": wk or "default", "pinned": a.pinned,
               "ms_per_call": el * 1e3,
               "votes_per_s": db.n / el, "wire_bytes": int(wire.size), "outputs_equal_device_soa_path": True}
        if a.trace and sp != "plain":
            with eng.options(host_trace=2):
                eng.validate_wire_proposals(wire, off, lens, scope, db.now)
            row["trace"] = eng.last_host_trace()
        print(json.dumps(row), flush=True)
    if a.device_walk:
        from hashgraph_like_consensus.device import DeviceWire
        dw = DeviceWire(np.asarray(wire), off, lens, scope, db.now)
        for _ in range(max(1, a.rounds)):
            for wk in a.device_walk.split(","):
                eng.set_option("wire_walk", {"lane": 0, "lds": 1}.get(wk, -1))
                eng.validate_wire_proposals_device(dw)
                torch.cuda.synchronize()
                assert np.array_equal(dw.results_numpy(), ref), wk
                t = time.perf_counter()
                for _ in range(a.steps):
                    eng.validate_wire_proposals_device(dw)
                torch.cuda.synchronize()
                el = (time.perf_counter() - t) / a.steps
                print(json.dumps({"device_resident_walk": wk, "ms_per_call": el * 1e3, "votes_per_s": db.n / el}),
                      flush=True)
        eng.set_option("wire_walk", -1)
    if arena is not None:
        arena.close()
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
