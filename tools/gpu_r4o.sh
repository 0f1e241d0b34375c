#!/bin/bash
# Cost-volume backward occupancy A/B (D = 32 kernel compiled for 2 / 3 / 4 waves per SIMD):
# microbench, then the train step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
for w in 2 3 4; do
  KDPC_CV_BWD_WPE=$w timeout -k 10 200 python -u tools/bench_cv_bwd.py > $O/r4o_cv_$w.log 2>&1 || { echo "STOP cv $w"; tail -5 $O/r4o_cv_$w.log; exit 1; }
  echo "wpe=$w"; cat $O/r4o_cv_$w.log | grep cross
done
for w in 2 3 2 3; do
  KDPC_CV_BWD_WPE=$w timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/r4o_bench_$w.log 2>&1 || { echo "STOP bench $w"; tail -5 $O/r4o_bench_$w.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/r4o_bench_$w.log') if l.startswith('{')][-1]); print('wpe=$w', d['ms_per_step'], d['kd_step']['ms_per_step'])"
done
echo "== done"
