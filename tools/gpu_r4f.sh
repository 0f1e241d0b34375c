#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -k "knn" > gpurun_out/r4f_knn.log 2>&1
rc=$?; tail -2 gpurun_out/r4f_knn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_cv_bwd.py > gpurun_out/r4f_cvbwd.log 2>&1
rc=$?; cat gpurun_out/r4f_cvbwd.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --sections knn --no-cpu-baseline > gpurun_out/r4f_knnbench.log 2>&1
rc=$?; tail -1 gpurun_out/r4f_knnbench.log | cut -c1-700; exit $rc
