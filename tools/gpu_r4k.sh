#!/bin/bash
# One-launch gradient pack / plan hand-over (kdpc_copy_segments) and the single step-counter
# buffer: graph tests, the copy kernel test, train + KD bench, a kernel trace of the train step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py::test_copy_segments tests/test_gpu_graph.py > $O/r4k_tests.log 2>&1 || { echo "STOP tests"; tail -30 $O/r4k_tests.log; exit 1; }
tail -2 $O/r4k_tests.log
timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/r4k_bench.log 2>&1 || { echo "STOP bench"; tail -5 $O/r4k_bench.log; exit 1; }
tail -1 $O/r4k_bench.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_r4k_train" -o run --output-format csv -- python3 "$R/bench.py" --sections train --steps 5 --warmup 2 --no-cpu-baseline > $O/kt_r4k_train.log 2>&1 || { echo "STOP kt"; tail -5 $O/kt_r4k_train.log; exit 1; }
echo "== done"
