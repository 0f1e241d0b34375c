#!/bin/bash
# Step-level profile: rocprofv3 kernel trace of the graphed bench step (per-kernel table of
# one steady-state step) and a torch.profiler attribution of the eager step to call sites.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-sp}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kt_$TAG" -o run --output-format csv -- python3 "$R/bench.py" --steps 4 --warmup 2 --no-cpu-baseline --measure-steps 0 > gpurun_out/kt_$TAG.log 2>&1 || { echo "STOP kt"; exit 1; }
f=$(find "$R/gpurun_out/kt_$TAG" -name "*kernel_trace.csv" | head -1)
python3 tools/step_kernels.py "$f" 3 pc_bwd_data 12 70 > gpurun_out/step_$TAG.txt && head -30 gpurun_out/step_$TAG.txt
timeout -k 10 400 python3 tools/torch_profile.py --out gpurun_out/torch_prof_$TAG.txt > gpurun_out/torch_prof_$TAG.log 2>&1 || { echo "STOP tp"; exit 1; }
echo "== done"
