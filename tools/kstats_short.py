"""Short per-kernel table of a rocprofv3 kernel_stats.csv: `python tools/kstats_short.py FILE
[TAG] [--filter SUBSTR] [--top N]` -> average and total microseconds per kernel."""
import csv
import re
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    flt = sys.argv[sys.argv.index("--filter") + 1] if "--filter" in sys.argv else None
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 4
    if flt is not None and flt in args:
        args.remove(flt)
    if str(top) in args[1:]:
        args.remove(str(top))
    rows = list(csv.DictReader(open(args[0])))
    if flt:
        rows = [r for r in rows if flt in r["Name"]]
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    tag = args[1] if len(args) > 1 else ""
    parts = []
    for r in rows[:top]:
        m = re.search(r"([A-Za-z_]\w*)(<[^(]*>)?\(", r["Name"].replace("(anonymous namespace)::", ""))
        name = (m.group(1) + (m.group(2) or "")) if m else r["Name"][:40]
        parts.append(f"{name[:34]} {float(r['AverageNs']) / 1e3:.1f}")
    print(f"{tag:8s}", " | ".join(parts))


if __name__ == "__main__":
    main()
