#!/bin/bash
# Wide cost volume workgroup targets: CV / model / graph / KD tests, microbench, step A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 700 $T tests/test_gpu_fused.py tests/test_gpu_model.py tests/test_gpu_graph.py tests/test_gpu_kd.py > $O/r4v_t.log 2>&1 || { echo "STOP t"; tail -30 $O/r4v_t.log; exit 1; }
tail -1 $O/r4v_t.log
timeout -k 10 120 python -u tools/bench_cv_wide.py || { echo "STOP mb"; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/r4v_b_$i.log 2>&1 || { echo "STOP b"; tail -5 $O/r4v_b_$i.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/r4v_b_$i.log') if l.startswith('{')][-1]); print('run $i', d['ms_per_step'], d['kd_step']['ms_per_step'])"
done
echo "== done"
