#!/bin/bash
# LDS-streamed cost-volume row sums: bitwise CV tests, CV microbench, train/KD bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_fused.py -k "cost_volume" > $O/r4p_t.log 2>&1 || { echo "STOP t"; tail -30 $O/r4p_t.log; exit 1; }
tail -1 $O/r4p_t.log
timeout -k 10 200 python -u tools/bench_cv_bwd.py > $O/r4p_cv.log 2>&1 || { echo "STOP cv"; tail -5 $O/r4p_cv.log; exit 1; }
grep cross $O/r4p_cv.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/r4p_bench_$i.log 2>&1 || { echo "STOP bench"; tail -5 $O/r4p_bench_$i.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/r4p_bench_$i.log') if l.startswith('{')][-1]); print('run $i', d['ms_per_step'], d['kd_step']['ms_per_step'])"
done
echo "== done"
