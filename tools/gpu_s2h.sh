#!/bin/bash
# Lean 3 / 4 waves-per-SIMD builds of the D=32 cost-volume backward (W1 fragments from LDS,
# no cross-query prefetch): parity under the knob, microbench, whole-step A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
KDPC_CV_BWD_WPE=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -k "cost_volume or cross or flow_embedding or reference" > $O/pytest_wpe3.log 2>&1
rc=$?; tail -2 $O/pytest_wpe3.log; [ $rc -eq 0 ] || exit $rc
for w in 2 3 4; do
  KDPC_CV_BWD_WPE=$w timeout -k 10 200 python -u tools/bench_cv_bwd.py --iters 20 > $O/cvb_wpe.log 2>&1 || { echo "STOP cvb $w"; tail -5 $O/cvb_wpe.log; exit 1; }
  echo "wpe=$w $(grep cross0 $O/cvb_wpe.log | cut -c1-200)"
done
run() {
  env "$@" timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/s2h_b.log 2>&1 || { echo "STOP $*"; tail -5 $O/s2h_b.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/s2h_b.log') if l.startswith('{')][-1]); print('$*', d['ms_per_step'], d['kd_step']['ms_per_step'])"
}
for rnd in 1 2 3; do
  run X=0
  run KDPC_CV_BWD_WPE=3
done
echo "== done"
