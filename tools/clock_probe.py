"""Shader clock under k_rec_main, measured per MI355X_MICROARCH.md 'DVFS give-back' item 6 (GPU box).

Run with a probe build (make variant NAME=clk DEFS=-DHLC_CLOCK_PROBE; HLC_LIB points at it): the
config-2 batch (640k votes, generated on the device) goes through hlc_validate_proposals_device
back to back for --seconds; then --last stamped launches are separated by marker lines.  Every
launch's k_rec_main blocks print `HLC_CLOCK block b votes v clk c wall w GHz g` (s_memtime ticks
over s_memrealtime ticks); `summarize` reads the log and reports, per variant, the median clock
of the last launch's blocks and the back-to-back votes/s.

    HLC_LIB=.../libhlc_clk.so python tools/clock_probe.py run --tag clk > gpurun_out/clk.log
    python tools/clock_probe.py summarize gpurun_out/clk*.log
"""
from __future__ import annotations

import argparse
import os
import re
import statistics
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
    for k in range(args.last):
        print(f"HLC_MARK {k}", flush=True)
        eng.validate_proposals_device(db, s.cuda_stream)
        torch.cuda.synchronize()
    print("HLC_END", flush=True)
    eng.close()


def summarize(paths) -> None:
    pat = re.compile(r"HLC_CLOCK block (\d+) votes (\d+) clk (\d+) wall (\d+) GHz ([\d.]+)")
    for p in paths:
        rate, cur, last = None, None, []
        for line in open(p, errors="replace"):
            if line.startswith("HLC_RATE"):
                rate = line.strip()
            elif line.startswith("HLC_MARK"):
                cur = []
            elif line.startswith("HLC_END"):
                last = cur or []
            else:
                m = pat.search(line)
                if m and cur is not None:
                    cur.append(float(m.group(5)))
        med = statistics.median(last) if last else float("nan")
        lo = min(last) if last else float("nan")
        hi = max(last) if last else float("nan")
        print(f"{os.path.basename(p)}: last stamped launch: {len(last)} blocks, median {med:.3f} GHz "
              f"(min {lo:.3f}, max {hi:.3f}); {rate}")


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
