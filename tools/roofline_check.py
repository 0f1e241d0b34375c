"""Cross-check bench.py's live roofline against a rocprofv3 --kernel-trace of the same command.

    python tools/roofline_check.py <rocprof dir with *kernel_trace.csv> <bench json line file>

For each roofline object in the bench line (the headline `roofline`, `kd_step.roofline`,
`configs1.*`, `roofline_knn`, ...): rocprof per-launch duration = the summed durations of its
entry's HIP kernels / launches of its first kernel, next to the live HIP-event average
(avg_launch_us).  Profile a single-section bench command (`--sections train`, `kd`,
`configs1` or `knn`): the rocprof sums cover every launch in the process, except for the
train / KD entries, which count the launches inside the measurement window bench.py marks
with two spin kernels (torch.cuda._sleep).
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


EXCLUDE = {"kdpc_knn_point": ("true>",)}  # knn_cull_kernel<QW, true>: the STATS variant


def main():
    import bench
    d, bench_file = sys.argv[1], sys.argv[2]
    line = None
    for ln in open(bench_file):  # the last JSON object line (a single-section run has no
        ln = ln.strip()           # "metric": its line holds only that section's record)
        if ln.startswith("{"):
            try:
                line = json.loads(ln)
            except ValueError:
                pass
    trace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(trace)))
    # bench.py brackets the train / KD sections' measurement steps with spin kernels: their
    # entries are compared on the launches inside that window only
    spins = sorted(int(x["Start_Timestamp"]) for x in rows if "spin_kernel" in x["Kernel_Name"])
    window = (spins[0], spins[-1]) if len(spins) >= 2 else None  # (bench also spins before
    # every bracketed launch: those lie inside the window)
    out = {}

    def objs(d, path):
        for k, v in d.items():
            if isinstance(v, dict):
                if "avg_launch_us" in v and v.get("kernel") in bench.ROOFLINE:
                    yield path + k, v
                yield from objs(v, path + k + ".")

    for key, r in objs(line or {}, ""):
        kernels = bench.ROOFLINE[r["kernel"]][3]
        sel = rows
        if window and key in ("roofline", "kd_step.roofline"):
            sel = [x for x in rows if window[0] < int(x["Start_Timestamp"]) < window[1]]
        wgs = r.get("grid_workgroups")
        if wgs:  # one entry timed at two shapes in one run (gather C=3 / C=64): by grid size
            sel = [x for x in rows if int(x["Grid_Size_X"]) * int(x["Grid_Size_Y"]) *
                   int(x["Grid_Size_Z"]) // max(1, int(x["Workgroup_Size_X"]) *
                   int(x["Workgroup_Size_Y"]) * int(x["Workgroup_Size_Z"])) == wgs]
        # the counting launch of the kNN evaluation count (kdpc_knn_point_evals) is not part
        # of the timed launches
        skip = EXCLUDE.get(r["kernel"], ())
        sel = [x for x in sel if not any(p in x["Kernel_Name"] for p in skip)]
        # launches of the entry = launches of the first of its kernels (list order) present
        head = next((k for k in kernels if any(k in x["Kernel_Name"] for x in sel)), kernels[0])
        n = sum(1 for x in sel if head in x["Kernel_Name"])
        tot = sum(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in sel
                  if any(k in x["Kernel_Name"] for k in kernels))
        rp = tot / max(n, 1) / 1e3
        out[key] = {"entry": r["kernel"], "hip_kernels": kernels, "rocprof_launches": n,
                    "rocprof_avg_us_per_launch": round(rp, 2),
                    "live_hip_event_avg_us": r["avg_launch_us"],
                    "ratio_live_over_rocprof": round(r["avg_launch_us"] / rp, 3) if rp else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
