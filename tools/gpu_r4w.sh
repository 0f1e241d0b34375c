#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for w in 512 256 1024 2048; do
  echo "target $w"; KDPC_PC_BWD_TARGET_WG=$w timeout -k 10 200 python -u tools/bench_pc_tiled.py 2>&1 | grep "untiled_us'" || { echo "STOP $w"; exit 1; }
done
echo "== done"
