"""Print a rocprofv3 kernel_stats.csv found under a directory: kernel, calls, average us."""
import csv
import glob
import re
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    m = re.search(r"::(k_\w+)[(<]", r["Name"])
    n = m.group(1) if m else r["Name"][:40]
    print(f"{n:42s} {r['Calls']:>4} avg {float(r['AverageNs']) / 1e3:10.1f} us")
