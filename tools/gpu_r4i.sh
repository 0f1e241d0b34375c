#!/bin/bash
# KD step: the student's decoder coordinate fork re-decided on an A/B (round 4)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
SECTIONS=kd BENCH_EXTRA="--mode kd --batch 4" TAG=kdf bash tools/gpu_bench_ab.sh off: on:KDPC_KD_COORD_FORK=1 own:KDPC_KD_COORD_FORK=1,KDPC_COORD_OWN_STREAM=1 off2: on2:KDPC_KD_COORD_FORK=1 own2:KDPC_KD_COORD_FORK=1,KDPC_COORD_OWN_STREAM=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k neg_sum > gpurun_out/r4i_ns.log 2>&1 || { tail -20 gpurun_out/r4i_ns.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread -k "cost_volume or reference_neighbours or layers_match or flow_layers or weightnet" > gpurun_out/r4i_cv.log 2>&1
rc=$?; tail -2 gpurun_out/r4i_cv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/entry_rooflines.py > gpurun_out/r4i_entry.log 2>&1
rc=$?; grep cost_volume gpurun_out/r4i_entry.log; exit $rc
