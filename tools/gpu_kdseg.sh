set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_kd.py -m gpu -x -q --timeout 250 --timeout-method thread -k "equals_eager or coordinate_fork or teacher_stream" > gpurun_out/kdseg_off.log 2>&1
rc=$?; echo "fork tests rc=$rc"; [ $rc -le 1 ] || exit $rc
tail -3 gpurun_out/kdseg_off.log
