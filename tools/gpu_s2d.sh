#!/bin/bash
# Pull-form cost-volume backward A/B: microbench under the kernel's knobs, then the step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"; TAG=${1:-s2d}
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 200 --timeout-method thread -k "pull or csr_bitwise" > $O/pytest_pull_$TAG.log 2>&1
rc=$?; tail -2 $O/pytest_pull_$TAG.log; [ $rc -eq 0 ] || exit $rc
for cfg in "X=0" "KDPC_CV_BWD_DIAG_NOROWS=1" "KDPC_CV_PULL_U=8" "KDPC_CV_PULL_XCD=1" "KDPC_CV_PULL_MORTON=1" "KDPC_CV_PULL_MORTON=1 KDPC_CV_PULL_XCD=1" "KDPC_CV_PULL_MORTON=1 KDPC_CV_PULL_XCD=1 KDPC_CV_PULL_U=8"; do
  env $cfg timeout -k 10 200 python -u tools/bench_cv_bwd.py --iters 30 > $O/cvb_$TAG.log 2>&1 || { echo "STOP cvb $cfg"; tail -5 $O/cvb_$TAG.log; exit 1; }
  echo "== $cfg"; grep cross $O/cvb_$TAG.log | sed -e "s/'bit_identical': True, //" -e "s/'pull_max_rel_dp2': [0-9.e-]*//"
done
echo "== done"
