set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export TMPDIR=/tmp
export KDPC_KD_COORD_FORK=1
export KDPC_COORD_OWN_STREAM=1
timeout -k 10 240 python -u tools/kd_capture_diag.py --seq --keep-events > gpurun_out/kdcap_own_keep.log 2>&1
rc=$?; echo "own-stream seq keep-events rc=$rc"; tail -40 gpurun_out/kdcap_own_keep.log; [ $rc -eq 0 ] || exit $rc
PYTHONPATH=tools timeout -k 10 300 python -u -m pytest -p no:faulthandler -p segv_plugin tests/test_gpu_graph.py tests/test_gpu_kd.py -m gpu -x -v --timeout 250 --timeout-method thread -k "equals_eager or coordinate_fork or teacher_stream" > gpurun_out/kdcap_own_pytest.log 2>&1
rc=$?; echo "own-stream pytest rc=$rc"; tail -70 gpurun_out/kdcap_own_pytest.log; exit $rc
