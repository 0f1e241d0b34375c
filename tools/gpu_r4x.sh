#!/bin/bash
# PointConv bias gradient from the weight kernel: tests, then train/KD A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 700 $T tests/test_gpu_fused.py tests/test_gpu_model.py tests/test_gpu_graph.py tests/test_gpu_kd.py > $O/r4x_t.log 2>&1 || { echo "STOP t"; tail -30 $O/r4x_t.log; exit 1; }
tail -1 $O/r4x_t.log
for v in 1 0 1 0; do
  KDPC_PC_BIAS_IN_WEIGHT=$v timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/r4x_b_$v.log 2>&1 || { echo "STOP b"; tail -5 $O/r4x_b_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/r4x_b_$v.log') if l.startswith('{')][-1]); print('bias_in_weight=$v', d['ms_per_step'], d['kd_step']['ms_per_step'])"
done
echo "== done"
