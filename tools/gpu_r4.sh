#!/bin/bash
# Round-4 GPU check: full pytest -m gpu (native backtrace on a crash), then a bench line.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-r4}
export TMPDIR=/tmp
PYTHONPATH=tools timeout -k 10 1000 python -u -m pytest -p no:faulthandler -p segv_plugin tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ]; then grep -n "FAILED\|Error\|native backtrace" gpurun_out/pytest_gpu_$TAG.log | head -20; exit $rc; fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
  rc=$?; tail -2 gpurun_out/bench_$TAG.log; exit $rc
fi
