#!/bin/bash
# Step profile: rocprofv3 kernel-trace stats of a short bench run + torch-profiler op view.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-step}
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --measure-steps 0 > gpurun_out/prof_$TAG.log 2>&1 || { echo "STOP rocprof"; exit 1; }
timeout -k 10 300 python tools/torch_profile.py > gpurun_out/torchprof.log 2>&1 || { echo "STOP torchprof"; exit 1; }
echo done
