#!/bin/bash
# Tiled PointConv backward A/B: kernel tests, then train+KD bench tiled / untiled, kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_fused.py -k "tiled or tile_plan" > $O/r4m_t1.log 2>&1 || { echo "STOP t1"; tail -40 $O/r4m_t1.log; exit 1; }
tail -1 $O/r4m_t1.log
for v in 1 0 1 0; do
  KDPC_PC_TILED=$v timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/r4m_bench_$v.log 2>&1 || { echo "STOP bench $v"; tail -5 $O/r4m_bench_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$O/r4m_bench_$v.log') if l.startswith('{')][-1]); print('tiled=$v', d['ms_per_step'], d['kd_step']['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_r4m_train" -o run --output-format csv -- python3 "$R/bench.py" --sections train --steps 5 --warmup 2 --no-cpu-baseline > $O/kt_r4m_train.log 2>&1 || { echo "STOP kt"; tail -5 $O/kt_r4m_train.log; exit 1; }
echo "== done"
