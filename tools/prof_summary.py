"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py: per-step time by kernel
family and the top kernels.  usage: python tools/prof_summary.py <dir with run_kernel_stats.csv> [steps]"""
import collections
import csv
import os
import sys

d = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
rows = list(csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))))


def family(n):
    for key, fam in (("Cijk", "gemm(tensile)"), ("pc_", "pointconv fused"), ("pointconv_contract", "pointconv contract"),
                     ("knn", "knn"), ("fps", "fps"), ("cost_volume", "cost volume"), ("slab_sum", "cost volume"),
                     ("csr", "group/csr"), ("group_rows", "group/csr"), ("rocprim", "group/csr"),
                     ("direct_copy", "copies"), ("copyBuffer", "copies"), ("CatArray", "copies"),
                     ("reduce_kernel", "torch reduce"), ("at::native", "torch elementwise"),
                     ("fillBuffer", "torch elementwise"), ("MIOpen", "batchnorm")):
        if key in n:
            return fam
    return "other"


fam = collections.Counter()
cnt = collections.Counter()
for r in rows:
    f = family(r["Name"])
    fam[f] += float(r["TotalDurationNs"]) / 1e6 / steps
    cnt[f] += int(r["Calls"]) / steps
print(f"total {sum(fam.values()):.2f} ms/step")
for k, v in fam.most_common():
    print(f"{v:7.2f} ms {cnt[k]:6.0f} launches  {k}")
print("top kernels:")
for r in rows[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:7.2f} ms/step n={int(r['Calls'])//steps:4d} "
          f"avg={float(r['AverageNs'])/1e3:8.1f}us {r['Name'][:100]}")
