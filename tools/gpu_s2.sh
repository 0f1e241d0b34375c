#!/bin/bash
# Round-4 second session: the pull-form cost-volume backward (targeted tests + microbench),
# then the full GPU suite and the bench line.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"; TAG=${1:-s2}
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 200 --timeout-method thread -k "pull or csr_bitwise" > $O/pytest_pull_$TAG.log 2>&1
rc=$?; tail -4 $O/pytest_pull_$TAG.log; [ $rc -eq 0 ] || exit $rc
if [ "${CV:-1}" = "1" ]; then
  timeout -k 10 200 python -u tools/bench_cv_bwd.py > $O/cvb_$TAG.log 2>&1 || { echo "STOP cvb"; tail -5 $O/cvb_$TAG.log; exit 1; }
  cat $O/cvb_$TAG.log
fi
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1
  rc=$?; tail -4 $O/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 500 python -u bench.py > $O/bench_$TAG.log 2>&1 || { echo "STOP bench"; tail -5 $O/bench_$TAG.log; exit 1; }
  tail -1 $O/bench_$TAG.log | cut -c1-300
  KDPC_CV_BWD_PULL=0 timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/bench_nopull_$TAG.log 2>&1 || { echo "STOP bench nopull"; tail -5 $O/bench_nopull_$TAG.log; exit 1; }
  tail -1 $O/bench_nopull_$TAG.log | cut -c1-300
  KDPC_CV_BWD_PULL_WIDE=1 timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/bench_pullwide_$TAG.log 2>&1 || { echo "STOP bench pullwide"; tail -5 $O/bench_pullwide_$TAG.log; exit 1; }
  tail -1 $O/bench_pullwide_$TAG.log | cut -c1-300
fi
echo "== done"
