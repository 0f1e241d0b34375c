#!/bin/bash
# Per-kernel times of the fused PointConv microbenchmark (rocprofv3 kernel trace).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pc}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/pct_$TAG" -o run --output-format csv -- python3 "$R/tools/bench_pointconv.py" ${PCARGS:-} > gpurun_out/pct_$TAG.log 2>&1 || { echo "STOP"; exit 1; }
grep -v amdgpu gpurun_out/pct_$TAG.log | grep "TFLOPs" || true
