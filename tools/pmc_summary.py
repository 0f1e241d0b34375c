"""Per-kernel averages of rocprofv3 --pmc passes: python tools/pmc_summary.py <dir with p*/>."""
import collections
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for p in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(p)):
        k = re.sub(r"^void \(anonymous namespace\)::", "", r["Kernel_Name"])
        k = k.split("((anonymous")[0].split("(int")[0][:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])] += 1
for k, v in agg.items():
    print(k)
    for c, val in sorted(v.items()):
        print("   %-28s %14.4g" % (c, val / cnt[(k, c)]))
    if "SQ_WAVE_CYCLES" in v:
        w = v["SQ_WAVE_CYCLES"]
        print("   -> WAIT_ANY %.2f  WAIT_INST_ANY %.2f  ACTIVE %.2f of wave-cycles" % (
            v["SQ_WAIT_ANY"] / w, v["SQ_WAIT_INST_ANY"] / w, v["SQ_ACTIVE_INST_ANY"] / w))
