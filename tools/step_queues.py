"""Per-queue view of graph-replayed training steps from a rocprofv3 --kernel-trace CSV.

    python tools/step_queues.py <run_kernel_trace.csv> [--marker fps_kernel<1024, 8] [--top 25]

Steps are cut at consecutive launches of a once-per-step marker kernel (default: the plan
fork's level-1 FPS).  For the median steady-state step it prints the step span, each
hardware queue's busy time (union of its kernel intervals) and kernel count, the union over
all queues, and per queue the kernels with the most time; then the time during which only
one queue was busy (the serial part of the step).
"""
import argparse
import collections
import csv


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for a, b in sorted(iv):
        if cur_e is None or a > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="fps_kernel<1024, 8")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"])
            for r in csv.DictReader(open(a.trace))]
    rows.sort()
    marks = [r[0] for r in rows if a.marker in r[2]]
    steps = []
    for t0, t1 in zip(marks, marks[1:]):
        seg = [r for r in rows if t0 <= r[0] < t1]
        steps.append((t1 - t0, t0, t1, seg))
    if not steps:
        raise SystemExit("no marker pairs")
    spans = sorted(s[0] for s in steps)
    print("step spans (ms):", " ".join(f"{s / 1e6:.2f}" for s, *_ in steps))
    med = spans[len(spans) // 2]
    span, t0, t1, seg = min(steps, key=lambda s: abs(s[0] - med))
    print(f"median step: {span / 1e6:.3f} ms, {len(seg)} launches, union busy "
          f"{union([(r[0], min(r[1], t1)) for r in seg]) / 1e6:.3f} ms")
    byq = collections.defaultdict(list)
    for r in seg:
        byq[r[3]].append(r)
    for q, rs in sorted(byq.items(), key=lambda kv: -len(kv[1])):
        busy = union([(r[0], min(r[1], t1)) for r in rs])
        last = max(r[1] for r in rs)
        print(f"queue {q}: {len(rs)} launches, busy {busy / 1e6:.3f} ms, "
              f"last end at +{(last - t0) / 1e6:.3f} ms")
        agg = collections.defaultdict(lambda: [0, 0])
        for s, e, n, _ in rs:
            k = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:70]
            agg[k][0] += 1
            agg[k][1] += e - s
        for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
            print(f"    {t / 1e3:9.1f} us {c:4d}x  {k}")
    # serial part: time covered by exactly one queue
    ev = []
    for s, e, n, q in seg:
        ev.append((s, 1, q))
        ev.append((min(e, t1), -1, q))
    ev.sort()
    active = collections.Counter()
    last_t, single = ev[0][0], collections.Counter()
    for t, d, q in ev:
        qs = [k for k, v in active.items() if v > 0]
        if len(qs) == 1:
            single[qs[0]] += t - last_t
        elif len(qs) == 0:
            single["idle"] += t - last_t
        last_t = t
        active[q] += d
    print("time with exactly one queue busy (per queue) / all idle:",
          {k: round(v / 1e6, 3) for k, v in single.items()})


if __name__ == "__main__":
    main()
