#!/bin/bash
# Model / graph / KD / fused GPU tests after a numerics-free backward change.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 700 $T tests/test_gpu_model.py tests/test_gpu_graph.py tests/test_gpu_kd.py tests/test_gpu_graph_dist.py tests/test_gpu_kernels.py -k "not knn_seeded" > $O/r4z_t.log 2>&1 || { echo "STOP t"; tail -30 $O/r4z_t.log; exit 1; }
tail -1 $O/r4z_t.log
echo "== done"
