#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_r4_measure.sh r04a || exit 1
PYTHONPATH=tools MALLOC_PERTURB_=165 timeout -k 10 300 python -u -m pytest -p no:faulthandler -p segv_plugin tests/test_gpu_graph.py tests/test_gpu_kd.py -m gpu -x -v --timeout 250 --timeout-method thread -k "equals_eager or coordinate_fork or teacher_stream" > gpurun_out/r4e_perturb.log 2>&1
rc=$?; echo "perturbed capture tests rc=$rc"; tail -12 gpurun_out/r4e_perturb.log; exit $rc
