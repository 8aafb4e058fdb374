"""Per-step timeline of the headline leg from a rocprofv3 kernel trace (tools/profile.sh trace/).

Each validate-many call launches k_rec_prep -> k_rec_main (second stream) and k_prehash_fused ->
k_chain_small (launch stream), then k_rec_comb -> k_rec_final -> k_rec_addr -> ... -> k_finalize
(round 6 on: k_rec_ucomb in k_rec_main's tail, then k_rec_add -> k_rec_final -> ...).
For the last --steps calls of the trace this prints the call span (first kernel start to
k_finalize end), the recovery's critical path (prep's duration + k_rec_main's start to k_rec_addr's
end), the gaps between call spans (host launch overhead), and the averages -- the
check that the chain's rocprof sum fits inside the bench line's ms_per_step.

    python tools/trace_steps.py profiles/r03_rocprof/trace/run_kernel_trace.csv --steps 20
"""
from __future__ import annotations

import argparse
import csv
import json
import re
import statistics

CHAIN_FUSED = ("k_rec_prep", "k_rec_main", "k_rec_comb", "k_rec_final", "k_rec_addr")
CHAIN_EARLY = ("k_rec_prep", "k_rec_main", "k_rec_ucomb", "k_rec_add", "k_rec_final", "k_rec_addr")


def short(name: str) -> str:
    m = re.search(r"::(k_\w+)[(<]", name)
    return m.group(1) if m else name[:40]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    rows = sorted(({"k": short(r["Kernel_Name"]), "s": int(r["Start_Timestamp"]), "e": int(r["End_Timestamp"])}
                   for r in csv.DictReader(open(a.trace))), key=lambda r: r["s"])
    CHAIN = CHAIN_EARLY if any(r["k"] == "k_rec_ucomb" for r in rows) else CHAIN_FUSED
    # calls are delimited by k_rec_prep launches (one per validate-many call)
    starts = [i for i, r in enumerate(rows) if r["k"] == "k_rec_prep"]
    calls = []
    for ci, i0 in enumerate(starts):
        i1 = starts[ci + 1] if ci + 1 < len(starts) else len(rows)
        ks = rows[max(0, i0 - 3):i1]  # the mapping kernels launched just before k_rec_prep
        byk = {}
        for r in ks:
            byk.setdefault(r["k"], r)
        if not all(k in byk for k in CHAIN) or "k_finalize" not in byk:
            continue
        t0 = min(r["s"] for r in ks if r["k"] in CHAIN + ("k_prehash_fused", "k_assign_props", "k_red_init"))
        calls.append({"t0": t0, "t1": byk["k_finalize"]["e"],
                      "chain_ms": (byk["k_rec_prep"]["e"] - byk["k_rec_prep"]["s"]
                                   + byk["k_rec_addr"]["e"] - byk["k_rec_main"]["s"]) / 1e6,
                      "kernels_ms": {k: (byk[k]["e"] - byk[k]["s"]) / 1e6 for k in CHAIN + ("k_prehash_fused",) if k in byk}})
    calls = calls[-a.steps:]
    if not calls:
        print("no complete calls found")
        return 1
    spans = [(c["t1"] - c["t0"]) / 1e6 for c in calls]
    period = [(calls[i + 1]["t0"] - calls[i]["t0"]) / 1e6 for i in range(len(calls) - 1)]
    out = {
        "calls": len(calls),
        "call_span_ms_mean": statistics.mean(spans),
        "step_period_ms_mean": statistics.mean(period) if period else None,
        "serial_recovery_chain_ms_mean": statistics.mean(c["chain_ms"] for c in calls),
        "kernel_ms_mean": {k: statistics.mean(c["kernels_ms"][k] for c in calls) for k in calls[0]["kernels_ms"]},
    }
    if a.json:
        print(json.dumps(out, indent=1))
    else:
        for k, v in out.items():
            print(f"{k}: {v}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
