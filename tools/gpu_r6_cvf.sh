#!/bin/bash
# Narrow cost-volume forward back on split-bf16: timing, the GPU tests it touches, and the
# graphed train step's reproducibility (two graphs side by side, tools/kd_race.py gg).
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/r6/$name.txt 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -E "RESULT|passed|failed|cross|us" gpurun_out/r6/$name.txt | tail -6
  [ $rc -eq 0 ] || { echo "STOP $name $rc"; grep -v "^frame" gpurun_out/r6/$name.txt | tail -8; exit $rc; }
}
step cvf_bench 200 python3 -u tools/bench_cv_fwd.py
step cvf_tests 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_kernels.py tests/test_gpu_graph.py tests/test_gpu_model.py
step gg_train 300 python3 -u tools/kd_race.py gg kind=train steps=24
step gg_kd 300 python3 -u tools/kd_race.py gg kind=kd tgraph=0 steps=24
