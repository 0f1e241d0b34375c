#!/bin/bash
# Lean D_IN=64 cost-volume forward (W1 from LDS, no cross-query prefetch; 3 waves per SIMD):
# outputs vs the default build (checksums), parity tests under the knob, whole-step A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
for l in 0 1; do
  KDPC_CV_FWD_LEAN=$l timeout -k 10 200 python -u tools/bench_cv_fwd.py > $O/cvf_$l.log 2>&1 || { echo "STOP cvf $l"; tail -5 $O/cvf_$l.log; exit 1; }
  echo "lean=$l"; grep cross $O/cvf_$l.log
done
KDPC_CV_FWD_LEAN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -k "cost_volume or cross or flow_embedding or reference" > $O/pytest_lean_fwd.log 2>&1
rc=$?; tail -2 $O/pytest_lean_fwd.log; [ $rc -eq 0 ] || exit $rc
run() {
  env "$@" timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/s2j_b.log 2>&1 || { echo "STOP $*"; tail -5 $O/s2j_b.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/s2j_b.log') if l.startswith('{')][-1]); print('$*', d['ms_per_step'], d['kd_step']['ms_per_step'])"
}
for rnd in 1 2 3; do
  run X=0
  run KDPC_CV_FWD_LEAN=1
done
echo "== done"
