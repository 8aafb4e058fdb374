"""Summarises tools/fetch_calib's two rocprofv3 passes (FETCH_SIZE, WRITE_SIZE): per access shape the
counter's bytes (KiB x 1024, averaged over the launches) over the bytes the kernel really touched --
the factor a profile's FETCH_SIZE / WRITE_SIZE must be divided by for kernels of that shape.

    python tools/fetch_calib.py <fetch_dir> <write_dir> <stdout-of-fetch_calib>
"""
import csv
import glob
import json
import os
import re
import sys


def per_kernel(d, counter):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    out = {}
    for p in path:
        with open(p, newline="") as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] != counter:
                    continue
                m = re.search(r"(k_\w+(?:<\d+>)?)", r["Kernel_Name"])
                if m:
                    out.setdefault(m.group(1), []).append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in out.items()}


def main():
    fdir, wdir, log = sys.argv[1:4]
    true = json.loads([l for l in open(log) if l.startswith("{")][-1])["bytes"]
    fetch, write = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    rows = {}
    for k, b in true.items():
        ctr = write.get(k) if k.startswith("k_write") else fetch.get(k)
        rows[k] = {"true_bytes": b, "counter": "WRITE_SIZE" if k.startswith("k_write") else "FETCH_SIZE",
                   "counter_bytes": ctr, "counter_over_true": (ctr / b) if ctr else None}
    print(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
