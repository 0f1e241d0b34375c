#!/bin/bash
# A/B of the PointConv backward kernels (KDPC_PC_WGT_WS=0/1): microbench times, bitwise
# comparison of every backward output, and a rocprofv3 kernel-trace of the flow0 shape.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ab}
if [ -n "${PRE:-}" ]; then
  timeout -k 10 300 bash -c "$PRE" > gpurun_out/pre_$TAG.log 2>&1 || { echo "STOP pre"; cat gpurun_out/pre_$TAG.log | tail -20; exit 1; }
  tail -40 gpurun_out/pre_$TAG.log
fi
KDPC_PC_WGT_WS=0 timeout -k 10 200 python -u tools/bench_pointconv.py --dump /tmp/pc_old.npz > gpurun_out/pc_old_$TAG.log 2>&1 || { echo "STOP old"; tail gpurun_out/pc_old_$TAG.log; exit 1; }
KDPC_PC_WGT_WS=1 timeout -k 10 200 python -u tools/bench_pointconv.py --dump /tmp/pc_new.npz > gpurun_out/pc_new_$TAG.log 2>&1 || { echo "STOP new"; tail gpurun_out/pc_new_$TAG.log; exit 1; }
echo "== old"; cat gpurun_out/pc_old_$TAG.log | grep -v amdgpu.ids
echo "== new"; cat gpurun_out/pc_new_$TAG.log | grep -v amdgpu.ids
python - <<'PY'
import numpy as np
a = np.load("/tmp/pc_old.npz"); b = np.load("/tmp/pc_new.npz")
for k in a.files:
    same = np.array_equal(a[k], b[k])
    d = float(np.abs(a[k].astype(np.float64) - b[k]).max()) if not same else 0.0
    print("bitwise" if same else "DIFF", k, a[k].shape, d)
PY
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kt_pc_$TAG" -o run --output-format csv -- python3 tools/bench_pointconv.py --only flow0 > gpurun_out/kt_pc_$TAG.log 2>&1 || { echo "STOP kt"; exit 1; }
f=$(find gpurun_out/kt_pc_$TAG -name "*kernel_stats.csv" | head -1)
head -12 "$f" | cut -c1-200
