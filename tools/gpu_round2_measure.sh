#!/bin/bash
# Bench line + rocprofv3 kernel-trace stats of a short run (per-step kernel table).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-r02}
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1 || { echo "STOP bench"; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-600
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kt_$TAG" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --measure-steps 0 ${BENCH_ARGS:-} > gpurun_out/kt_$TAG.log 2>&1 || { echo "STOP kt"; exit 1; }
echo "== done"
