"""Shader clock under k_rec_main, measured per MI355X_MICROARCH.md 'DVFS give-back' item 6 (GPU box).

The config-2 batch (640k votes, generated on the device) goes through hlc_validate_proposals_device
back to back for --seconds; then --last calls run with the library's clock stamps on
(hlc_ctx_set_clock_probe: every k_rec_main wave stamps s_memtime / s_memrealtime at its start and end)
and each prints `HLC_CLOCK call k median m min a max b waves w`.  `summarize` reads the logs and
reports, per log, the last stamped call's clock and the back-to-back votes/s.  (HLC_LIB selects another
build of the library for an A/B.)

    python tools/clock_probe.py run --tag shipped > gpurun_out/clk.log
    python tools/clock_probe.py summarize gpurun_out/clk*.log
"""
from __future__ import annotations

import argparse
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hashgraph-like-consensus_amd", "python"))


def run(args) -> None:
    import torch

    from hashgraph_like_consensus import synth
    from hashgraph_like_consensus.device import DeviceBatch
    from hashgraph_like_consensus.engine import Engine

    eng = Engine(0)
    db = DeviceBatch.synthetic(eng, args.proposals, 64, 64, True, synth.config_seed(2), device="cuda:0")
    eng.reserve(db.n, args.proposals, db.bytes_len)
    s = torch.cuda.Stream(device="cuda:0")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    calls = 0
    while time.perf_counter() - t0 < args.seconds:
        for _ in range(20):
            eng.validate_proposals_device(db, s.cuda_stream)
        calls += 20
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"HLC_RATE tag={args.tag} calls={calls} seconds={el:.3f} votes_per_s={db.n * calls / el:.6g}", flush=True)
    eng.set_clock_probe(True)
    for k in range(args.last):
        eng.validate_proposals_device(db, s.cuda_stream)
        torch.cuda.synchronize()
        c = eng.clock_probe()
        print(f"HLC_CLOCK call {k} median {c['median_GHz']:.4f} min {c['min_GHz']:.4f} max {c['max_GHz']:.4f} "
              f"waves {c['waves']}", flush=True)
    eng.set_clock_probe(False)
    eng.close()


def summarize(paths) -> None:
    pat = re.compile(r"HLC_CLOCK call (\d+) median ([\d.]+) min ([\d.]+) max ([\d.]+) waves (\d+)")
    for p in paths:
        rate, last = None, None
        for line in open(p, errors="replace"):
            if line.startswith("HLC_RATE"):
                rate = line.strip()
            m = pat.search(line)
            if m:
                last = m
        if last is None:
            print(f"{os.path.basename(p)}: no stamped call; {rate}")
            continue
        print(f"{os.path.basename(p)}: last stamped call: {last.group(5)} waves, median {float(last.group(2)):.3f} GHz "
              f"(min {float(last.group(3)):.3f}, max {float(last.group(4)):.3f}); {rate}")


def main() -> int:
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--tag", default="clk")
    r.add_argument("--seconds", type=float, default=3.0)
    r.add_argument("--last", type=int, default=2)
    r.add_argument("--proposals", type=int, default=10_000)
    sm = sub.add_parser("summarize")
    sm.add_argument("paths", nargs="+")
    a = ap.parse_args()
    if a.cmd == "run":
        run(a)
    else:
        summarize(a.paths)
    return 0


if __name__ == "__main__":
    sys.exit(main())
