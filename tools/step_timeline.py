"""Per-step GPU timeline from a rocprofv3 --kernel-trace CSV: step boundaries at the first
kernel of each step (marker kernel's k-th launch), busy time (union of kernel intervals),
idle gaps, launch count and the biggest gaps.
usage: python tools/step_timeline.py <run_kernel_trace.csv> [marker substring] [launches of
       the marker per step]"""
import csv
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "pc_bwd_data_kernel"
per = int(sys.argv[3]) if len(sys.argv) > 3 else 12
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"])
        for r in csv.DictReader(open(path))]
rows.sort()
marks = [i for i, r in enumerate(rows) if marker in r[2]]
# a step ends at the last marker launch of its group
ends = [marks[k] for k in range(per - 1, len(marks), per)]
prev = None
for s, e in enumerate(ends):
    lo = 0 if prev is None else prev + 1
    seg = rows[lo:e + 1]
    prev = e
    if s == 0:
        continue
    t0, t1 = seg[0][0], max(r[1] for r in seg)
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for a, b, n, st in seg:
        if cur_e is None or a > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append((a - cur_e, n))
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    busy += cur_e - cur_s
    span = t1 - t0
    gaps.sort(reverse=True)
    small = sum(g for g, _ in gaps if g < 20000)
    print(f"step {s}: span {span/1e6:.2f} ms, busy {busy/1e6:.2f} ms, idle {(span-busy)/1e6:.2f} ms "
          f"({len(gaps)} gaps, {small/1e6:.2f} ms in gaps <20us), {len(seg)} launches")
    for g, n in gaps[:6]:
        print(f"     gap {g/1e3:8.1f} us before {n[:90]}")
