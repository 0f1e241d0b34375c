#!/bin/bash
# Final run of the session: full GPU suite, then the measurement pass (bench line, kernel
# traces + roofline cross-checks of the train and KD steps).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"; TAG=${1:-s2f}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -3 $O/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || exit $rc
PARTS=bench,kt SECS="train kd" bash tools/gpu_r4_measure.sh $TAG
