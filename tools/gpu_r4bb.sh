#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for w in 4096 2048 4096 2048; do
  echo "win $w"; KDPC_CV_SUM_WIN=$w timeout -k 10 200 python -u tools/bench_cv_bwd.py | grep cross || { echo STOP; exit 1; }
done
echo "== done"
