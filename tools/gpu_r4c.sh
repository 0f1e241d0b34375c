#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -p no:faulthandler -p segv_plugin -m gpu -x -v --timeout 200 --timeout-method thread"
export PYTHONPATH=tools
timeout -k 10 200 $PT tests/test_gpu_graph.py -k "joins_forked" > gpurun_out/r4c_guard.log 2>&1
rc=$?; tail -3 gpurun_out/r4c_guard.log; [ $rc -eq 0 ] || { grep -n "native backtrace" -A 30 gpurun_out/r4c_guard.log | head -40; exit $rc; }
timeout -k 10 900 $PT tests/test_gpu_model.py tests/test_gpu_graph.py tests/test_gpu_fused.py tests/test_gpu_kd.py tests/test_gpu_graph_dist.py > gpurun_out/r4c_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r4c_tests.log; grep -n "gradient error vs float64\|FAILED" gpurun_out/r4c_tests.log | head; [ $rc -eq 0 ] || exit $rc
for c in joined unjoined; do
  timeout -k 5 120 python -u tools/torch_unjoined_capture.py $c > gpurun_out/r4c_torch_$c.log 2>&1
  rc=$?; echo "torch capture $c rc=$rc"; tail -25 gpurun_out/r4c_torch_$c.log; [ $rc -eq 0 ] || break
done
timeout -k 10 300 $PT tests/test_gpu_kernels.py -k "knn or gather" > gpurun_out/r4c_knn.log 2>&1
rc=$?; tail -3 gpurun_out/r4c_knn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --sections knn,configs1 --no-cpu-baseline > gpurun_out/r4c_bench_knn.log 2>&1
rc=$?; tail -1 gpurun_out/r4c_bench_knn.log | cut -c1-3000; exit $rc
