"""Kernel time of ONE steady-state step from a rocprofv3 kernel trace, grouped by kernel
name (launches, total us), using the same step segmentation as step_timeline.py.
usage: python tools/step_kernels.py <run_kernel_trace.csv> [step index] [marker] [per]"""
import collections
import csv
import re
import sys

path = sys.argv[1]
which = int(sys.argv[2]) if len(sys.argv) > 2 else 2
marker = sys.argv[3] if len(sys.argv) > 3 else "pc_bwd_data_kernel"
per = int(sys.argv[4]) if len(sys.argv) > 4 else 12
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
              for r in csv.DictReader(open(path)))
marks = [i for i, r in enumerate(rows) if marker in r[2]]
ends = [marks[k] for k in range(per - 1, len(marks), per)]
seg = rows[ends[which - 1] + 1:ends[which] + 1]
agg = collections.defaultdict(lambda: [0, 0.0])
for a, b, n in seg:
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"rocprim::ROCPRIM_\w+::detail::", "rocprim::", n)
    key = n.split("(")[0][:90]
    agg[key][0] += 1
    agg[key][1] += (b - a) / 1e3
tot = sum(v[1] for v in agg.values())
print(f"step {which}: {len(seg)} launches, {tot/1e3:.2f} ms kernel time")
for k, (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[5]) if len(sys.argv) > 5 else 60]:
    print(f"{us:9.1f} us {c:5d}  {k}")
