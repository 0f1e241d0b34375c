#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for w in 512 256 1024 2048; do
  KDPC_CVW_WGS=$w timeout -k 10 120 python -u tools/bench_cv_wide.py || { echo "STOP $w"; exit 1; }
done
echo "== done"
