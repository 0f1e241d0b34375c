#!/bin/bash
# Kernel trace of the PointConv microbenchmark (flow0 only) for each diagnostic variant.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in base "$@"; do
  if [ $v = base ]; then unset KDPC_LIB; else export KDPC_LIB=$R/tools/variants/$v/libkdpc_hip.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/vt_$v" -o run --output-format csv -- python3 "$R/tools/bench_pointconv.py" --only flow0 --iters 5 > gpurun_out/vt_$v.log 2>&1 || { echo "STOP $v"; exit 1; }
  python3 - "$R/gpurun_out/vt_$v/run_kernel_stats.csv" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "pc_bwd" in r["Name"] or "pc_fwd" in r["Name"]:
        print(sys.argv[2], "%8.1f us" % (float(r["AverageNs"]) / 1e3), r["Name"][27:70])
PY
done
