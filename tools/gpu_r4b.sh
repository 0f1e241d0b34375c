#!/bin/bash
# capture-repro cases + gather parity + configs1 microbench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in torch_pattern event_two_streams side_forks_side event_outlives_capture stream_destroyed_in_capture unjoined side_forks_side_unjoined; do
  MALLOC_PERTURB_=165 timeout -k 5 60 tools/hip_capture_repro $c > gpurun_out/repro_$c.log 2>&1
  rc=$?; echo "repro $c rc=$rc"; cat gpurun_out/repro_$c.log
  if [ $rc -ne 0 ]; then echo "STOP after repro crash"; break; fi
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gather" > gpurun_out/pytest_gather.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gather.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --sections configs1,gather_c3,gather_c64 --no-cpu-baseline > gpurun_out/bench_cfg1.log 2>&1
rc=$?; tail -1 gpurun_out/bench_cfg1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['configs1']; [print(k, c[k]['avg_launch_us'], c[k]['frac']) for k in ('grouping_operation','gather_operation_c3','gather_operation_c64')]; [print(k, d[k]['avg_launch_us'], d[k]['frac']) for k in ('gather_c3','gather_c64')]"
true
[ $rc -eq 0 ] || exit $rc
TAG=cvw bash tools/gpu_bench_ab.sh base: wide:KDPC_CV_WIDE_FUSED=1 base2: wide2:KDPC_CV_WIDE_FUSED=1
