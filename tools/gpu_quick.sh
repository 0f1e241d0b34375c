#!/bin/bash
# Quick GPU iteration: parity subset + microbench + torch-profiler attribution.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_kernels.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_kernels.log; [ $rc -eq 0 ] || { echo "STOP pytest $rc"; exit $rc; }
timeout -k 10 300 python tools/microbench_ops.py --json gpurun_out/microbench.json > gpurun_out/mb.log 2>&1 || { echo "STOP mb"; exit 1; }
if [ "${TORCHPROF:-0}" = "1" ]; then
  timeout -k 10 300 python tools/torch_profile.py > gpurun_out/torchprof.log 2>&1 || { echo "STOP tprof"; exit 1; }
fi
echo ok
