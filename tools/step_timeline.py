"""Print one bench step's kernel timeline from a rocprofv3 kernel-trace CSV (start / end / duration in
us relative to the step's k_prehash_fused, queue, kernel, grid), plus every step's length.
  python tools/step_timeline.py TRACE.csv [STEP_INDEX]"""
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))

    def nm(s):
        m = re.search(r"(k_\w+|__amd\w+)", s)
        return m.group(1) if m else s[:30]

    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm(r["Kernel_Name"]), r["Queue_Id"],
                 int(r["Grid_Size_X"])) for r in rows)
    idx = [i for i, k in enumerate(ks) if k[2] == "k_prehash_fused"]
    print("step lengths (us):", " ".join(f"{(ks[b][0] - ks[a][0]) / 1e3:.0f}" for a, b in zip(idx, idx[1:])))
    j = int(sys.argv[2]) if len(sys.argv) > 2 else len(idx) - 2
    i0, i1 = idx[j], idx[j + 1]
    t0 = ks[i0][0]
    for k in ks[i0:i1 + 1]:
        print(f"{(k[0] - t0) / 1e3:9.1f} {(k[1] - t0) / 1e3:9.1f} {(k[1] - k[0]) / 1e3:8.1f} q{k[3]} {k[2]:30s} grid={k[4]}")


if __name__ == "__main__":
    main()
