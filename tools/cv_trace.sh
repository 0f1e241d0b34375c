#!/bin/bash
# Kernel trace of the cost-volume microbenchmark (tools/bench_cost_volume.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-cv}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/cvt_$TAG" -o run --output-format csv -- python3 "$R/tools/bench_cost_volume.py" --iters 5 > gpurun_out/cvt_$TAG.log 2>&1 || { echo "STOP"; exit 1; }
grep level gpurun_out/cvt_$TAG.log || true
python3 - "$R/gpurun_out/cvt_$TAG/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "cost_volume" in r["Name"] or "colsum" in r["Name"]:
        print("%8.1f us x%4s %s" % (float(r["AverageNs"]) / 1e3, r["Calls"], r["Name"][:80]))
PY
