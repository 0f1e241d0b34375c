"""HBM traffic per entry-point launch from rocprofv3 --pmc passes of bench.py.

    python tools/pmc_traffic.py --workload train_b8_n8192 --fetch <dir of FETCH_SIZE pass>
                                --write <dir of WRITE_SIZE pass> [--out profiles/pmc_traffic.json]
                                [--command "<the bench command both passes profiled>"]

Each pass is its own `rocprofv3 --pmc <counter> --output-format csv` run of the same bench
command (gfx950 cannot hold FETCH_SIZE and WRITE_SIZE in one pass).  Per
MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB, and on gfx950 FETCH_SIZE reports
1/2 of the bytes of a wide coalesced read, so hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024.
The per-launch figure of a C entry point sums its HIP kernels (bench.ROOFLINE) and divides by
the number of launches of the entry's first kernel.  Each pass must profile ONE workload (a
single-section bench command, e.g. `bench.py --sections kd`); the result is merged into the
output file under workloads[<workload>], the key bench.py looks traffic up by, so a figure is
never attached to a roofline of another workload.
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(d, counter):
    """-> {kernel short name: (dispatches, summed counter value)}"""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per_dispatch = {}
    for fn in files:
        for r in csv.DictReader(open(fn)):
            if r["Counter_Name"] != counter:
                continue
            key = (r.get("Agent_Id", ""), r["Dispatch_Id"])
            name = r["Kernel_Name"]
            v = float(r["Counter_Value"])
            prev = per_dispatch.get(key, (name, 0.0))
            per_dispatch[key] = (name, prev[1] + v)
    out = collections.defaultdict(lambda: [0, 0.0])
    for name, v in per_dispatch.values():
        out[name][0] += 1
        out[name][1] += v
    return out


def match(name, short):
    return short in name


def main():
    import bench
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", required=True,
                    help="bench workload key (bench.workload_key / the section's `workload`)")
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--command", default="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline")
    args = ap.parse_args()
    fetch = load(args.fetch, "FETCH_SIZE")
    write = load(args.write, "WRITE_SIZE")
    entries = {}
    for entry, (_, _, _, kernels) in bench.ROOFLINE.items():
        if not kernels:
            continue
        head = kernels[0]
        # an entry whose kernels are a strict subset of another entry's with the same first
        # kernel (kdpc_cost_volume_bwd inside kdpc_cost_volume_bwd_csr) cannot be told apart
        # by kernel name: its launches are the larger entry's, so it gets no figure of its own
        if any(e != entry and ks and ks[0] == head and set(kernels) < set(ks)
               for e, (_, _, _, ks) in bench.ROOFLINE.items()):
            continue
        launches = sum(n for name, (n, _) in fetch.items() if match(name, head))
        if launches == 0:
            continue
        fkb = sum(v for name, (_, v) in fetch.items() if any(match(name, k) for k in kernels))
        wkb = sum(v for name, (_, v) in write.items() if any(match(name, k) for k in kernels))
        entries[entry] = {
            "launches": launches,
            "fetch_size_kib_per_launch": fkb / launches,
            "write_size_kib_per_launch": wkb / launches,
            "hbm_bytes_per_launch": round((2 * fkb + wkb) * 1024 / launches),
            "kernels": kernels,
        }
    try:
        with open(args.out) as f:
            res = json.load(f)
    except (OSError, ValueError):
        res = {}
    res["formula"] = "(2*FETCH_SIZE + WRITE_SIZE) * 1024 per launch (MI355X_MICROARCH.md §HBM)"
    res.setdefault("workloads", {})[args.workload] = {"command": args.command,
                                                      "entries": entries}
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res["workloads"][args.workload], indent=1))


if __name__ == "__main__":
    main()
