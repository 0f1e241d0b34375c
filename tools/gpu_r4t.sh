#!/bin/bash
# Cost-volume forward queries-per-wave A/B (outputs must not change: checksums printed).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for q in 8 16 32 64 4; do
  KDPC_CV_FWD_QPW=$q timeout -k 10 120 python -u tools/bench_cv_fwd.py || { echo "STOP $q"; exit 1; }
done
echo "== done"
