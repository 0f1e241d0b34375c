#!/bin/bash
# Tiled forward: kernel tests (bit-identical), model/graph tests, train/KD A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_fused.py -k "tiled" > $O/r4s_t1.log 2>&1 || { echo "STOP t1"; tail -30 $O/r4s_t1.log; exit 1; }
tail -1 $O/r4s_t1.log
timeout -k 10 600 $T tests/test_gpu_model.py tests/test_gpu_graph.py > $O/r4s_t2.log 2>&1 || { echo "STOP t2"; tail -30 $O/r4s_t2.log; exit 1; }
tail -1 $O/r4s_t2.log
for v in 1 0 1 0; do
  KDPC_PC_TILED_FWD=$v timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/r4s_b_$v.log 2>&1 || { echo "STOP b $v"; tail -5 $O/r4s_b_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/r4s_b_$v.log') if l.startswith('{')][-1]); print('tiled_fwd=$v', d['ms_per_step'], d['kd_step']['ms_per_step'])"
done
echo "== done"
