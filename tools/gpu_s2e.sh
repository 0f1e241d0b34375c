#!/bin/bash
# Cost-volume backward: batch-chunked plain / ranked paths (microbench), then the default step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"; TAG=${1:-s2e}
timeout -k 10 300 python -u tools/bench_cv_bwd.py --iters 20 > $O/cvb_$TAG.log 2>&1 || { echo "STOP cvb"; tail -5 $O/cvb_$TAG.log; exit 1; }
grep cross $O/cvb_$TAG.log | sed -e "s/'bit_identical': True, //"
echo "== done"
