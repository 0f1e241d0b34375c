#!/bin/bash
# Round measurement: bench line, rocprofv3 kernel-trace of the same command (cross-check of
# the live roofline), and the two PMC passes for HBM traffic.  Each GPU step time-limited;
# any failure stops the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-r01}
export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline"
timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup 3 > gpurun_out/bench_$TAG.log 2>&1 || { echo "STOP bench"; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kt_$TAG" -o run --output-format csv -- $CMD > gpurun_out/kt_$TAG.log 2>&1 || { echo "STOP kt"; exit 1; }
grep '"metric"' gpurun_out/kt_$TAG.log > gpurun_out/kt_bench_$TAG.json
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "pc_|group_rows|group_points|cost_volume_|idw_" -d "$R/gpurun_out/pmcf_$TAG" -o run --output-format csv -- $CMD > gpurun_out/pmcf_$TAG.log 2>&1 || { echo "STOP pmc fetch"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "pc_|group_rows|group_points|cost_volume_|idw_" -d "$R/gpurun_out/pmcw_$TAG" -o run --output-format csv -- $CMD > gpurun_out/pmcw_$TAG.log 2>&1 || { echo "STOP pmc write"; exit 1; }
echo "== done"
