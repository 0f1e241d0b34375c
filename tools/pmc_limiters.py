"""Per-kernel limiter summary from rocprofv3 --pmc passes (one directory per pass).

    python tools/pmc_limiters.py <dir holding p1/ p2/ ...> [--out summary.json]

Per kernel (averaged over its dispatches) it prints the raw counters and these derived
figures (units per MI355X_MICROARCH.md §rocprofv3 PMC slots / §Per-instruction cycle
constants):
  cycles           GRBM_GUI_ACTIVE / 8          (the counter sums the 8 XCDs)
  mfma_busy        SQ_VALU_MFMA_BUSY_CYCLES / (cycles * 1024 SIMDs)
  wave_slots       SQ_WAVE_CYCLES * 4 / (cycles * 1024)   (mean resident waves per SIMD;
                   the SQ wave counters tick in quad-cycles)
  wait_any / wait_inst_any / active_any   SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY as
                   fractions of SQ_WAVE_CYCLES (parked on waitcnt/barrier, issue-stalled,
                   issuing: disjoint)
  valu_per_mfma, lds_per_mfma, vmem_per_mfma   instruction mix
  lds_conflict     SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  l2_hit           TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  hbm_bytes        (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving)
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def short(name):
    k = re.sub(r"^void ", "", name)
    k = re.sub(r"\(anonymous namespace\)::", "", k)
    return k.split("(")[0][:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    a = ap.parse_args()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(set))
    for fn in sorted(glob.glob(os.path.join(a.dir, "p*", "**", "*counter_collection.csv"),
                           recursive=True)):
        pdir = fn[len(a.dir):].lstrip("/").split("/")[0]
        for r in csv.DictReader(open(fn)):
            k = short(r["Kernel_Name"])
            c = r["Counter_Name"]
            per[k][c] += float(r["Counter_Value"])
            cnt[k][c].add((pdir, r.get("Agent_Id", ""), r["Dispatch_Id"]))
    res = {}
    for k, v in per.items():
        m = {c: val / max(1, len(cnt[k][c])) for c, val in v.items()}
        d = {}
        cyc = m.get("GRBM_GUI_ACTIVE", 0.0) / 8
        if cyc:
            d["cycles"] = cyc
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                d["mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024)
            if "SQ_WAVE_CYCLES" in m:
                d["wave_slots"] = m["SQ_WAVE_CYCLES"] * 4 / (cyc * 1024)
        w = m.get("SQ_WAVE_CYCLES")
        if w:
            for c, n in (("SQ_WAIT_ANY", "wait_any"), ("SQ_WAIT_INST_ANY", "wait_inst_any"),
                         ("SQ_ACTIVE_INST_ANY", "active_any"), ("SQ_WAIT_INST_LDS", "wait_inst_lds"),
                         ("SQ_ACTIVE_INST_VALU", "active_valu"), ("SQ_ACTIVE_INST_LDS", "active_lds")):
                if c in m:
                    d[n] = m[c] / w
        mf = m.get("SQ_INSTS_MFMA")
        if mf:
            for c, n in (("SQ_INSTS_VALU", "valu_per_mfma"), ("SQ_INSTS_LDS", "lds_per_mfma"),
                         ("SQ_INSTS_VMEM_RD", "vmem_rd_per_mfma"), ("SQ_INSTS_SALU", "salu_per_mfma")):
                if c in m:
                    d[n] = m[c] / mf
        if m.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_conflict"] = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_LDS_IDX_ACTIVE"]
        if "TCC_HIT_sum" in m and (m["TCC_HIT_sum"] + m.get("TCC_MISS_sum", 0)):
            d["l2_hit"] = m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m.get("TCC_MISS_sum", 0))
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            d["hbm_bytes"] = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
        res[k] = {"dispatches": max(len(s) for s in cnt[k].values()), "derived": d,
                  "counters": m}
    for k in sorted(res, key=lambda x: -res[x]["derived"].get("cycles", 0)):
        d = res[k]["derived"]
        print(k, res[k]["dispatches"])
        print("   " + "  ".join(f"{n}={v:.3g}" for n, v in d.items()))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
