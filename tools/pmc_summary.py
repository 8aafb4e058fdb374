#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 PMC passes (tools/profile.sh output): one line per kernel and
counter, averaged over its launches.  Usage: pmc_summary.py <prof dir> [kernel-substring ...]"""
import collections
import csv
import os
import re
import sys


def kernel_short(name: str) -> str:
    m = re.search(r"::(k_\w+)[(<]", name)
    return m.group(1) if m else name.split("(")[0][-40:]


def summarize(d: str, only=()):
    out = collections.defaultdict(dict)
    for sub in sorted(os.listdir(d)):
        f = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            acc[kernel_short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in acc.items():
            if only and not any(o in k for o in only):
                continue
            for c, v in cs.items():
                out[k][c] = (sum(v) / len(v), len(v))
    return out


if __name__ == "__main__":
    res = summarize(sys.argv[1], sys.argv[2:])
    for k in sorted(res):
        print(k, " ".join(f"{c}={v:.4g}(x{n})" for c, (v, n) in sorted(res[k].items())))
