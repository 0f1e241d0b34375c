#!/bin/bash
# Round 6: the packed-f32 fix against every race diagnostic, then the KD / graph GPU tests.
# Each step under its own limit; stop at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
step() {  # name limit command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/r6/$name.txt 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -E "RESULT|passed|failed|twice:" gpurun_out/r6/$name.txt | tail -4
  [ $rc -eq 0 ] || { echo "STOP $name $rc"; grep -v "^frame" gpurun_out/r6/$name.txt | tail -8; exit $rc; }
}
step knn_twice 200 python3 -u tools/knn_race.py shapes=model main=teacher twice=1 reps=600
step knn_twice_eager 200 python3 -u tools/knn_race.py shapes=model main=teacher twice=1 eager=1 reps=300
step fwd_tt 200 python3 -u tools/fwd_race.py tt reps=300
step gg_kd 300 python3 -u tools/kd_race.py gg kind=kd steps=24
step gg_kd_onegraph 300 python3 -u tools/kd_race.py gg kind=kd tgraph=0 steps=24
step pytest_kd_graph 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kd.py tests/test_gpu_graph.py
