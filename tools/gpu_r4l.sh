#!/bin/bash
# Tiled PointConv backward: kernel tests, model / graph / KD tests, train + KD bench, and a
# kernel trace of the train step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_fused.py -k "tiled or tile_plan or pointconv" > $O/r4l_t1.log 2>&1 || { echo "STOP t1"; tail -40 $O/r4l_t1.log; exit 1; }
tail -1 $O/r4l_t1.log
timeout -k 10 600 $T tests/test_gpu_model.py tests/test_gpu_graph.py tests/test_gpu_kd.py > $O/r4l_t2.log 2>&1 || { echo "STOP t2"; tail -40 $O/r4l_t2.log; exit 1; }
tail -1 $O/r4l_t2.log
timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/r4l_bench.log 2>&1 || { echo "STOP bench"; tail -5 $O/r4l_bench.log; exit 1; }
tail -1 $O/r4l_bench.log | cut -c1-300
KDPC_PC_TILED=0 timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/r4l_bench_off.log 2>&1 || { echo "STOP bench off"; tail -5 $O/r4l_bench_off.log; exit 1; }
tail -1 $O/r4l_bench_off.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_r4l_train" -o run --output-format csv -- python3 "$R/bench.py" --sections train --steps 5 --warmup 2 --no-cpu-baseline > $O/kt_r4l_train.log 2>&1 || { echo "STOP kt"; tail -5 $O/kt_r4l_train.log; exit 1; }
echo "== done"
