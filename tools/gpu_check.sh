#!/bin/bash
# GPU-box check: parity tests, a short bench, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/abort/timeout stops the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-r01}
STEPS=${STEPS:-5}

ok_or_stop() {  # $1 = exit code; 0/1 (pytest pass/fail) continue, anything else stops
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: exit $1"; exit "$1"; fi
}

echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu_$TAG.log; ok_or_stop $rc

echo "== bench"
timeout -k 10 600 python bench.py --steps $STEPS --warmup 2 > gpurun_out/bench_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/bench_$TAG.log; [ $rc -eq 0 ] || { echo "STOP bench $rc"; exit $rc; }

if [ "${PROFILE:-1}" = "1" ]; then
  echo "== rocprofv3"
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run \
      --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/prof_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/prof_$TAG.log; [ $rc -eq 0 ] || { echo "STOP prof $rc"; exit $rc; }
  find "$R/gpurun_out/prof_$TAG" -name "*kernel_stats.csv" | head -3
fi
echo "== done"
