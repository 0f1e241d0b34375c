"""Print per-kernel average times from a rocprofv3 kernel_stats.csv:
python tools/kstats.py <run_kernel_stats.csv> [name substring ...]"""
import csv
import sys

pats = sys.argv[2:]
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if not pats or any(p in r["Name"] for p in pats):
        print("%9.1f us x%5s %s" % (float(r["AverageNs"]) / 1e3, r["Calls"], r["Name"][:90]))
