#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in external_event_kept; do
  MALLOC_PERTURB_=165 timeout -k 5 60 tools/hip_capture_repro $c > gpurun_out/repro_$c.log 2>&1
  rc=$?; echo "repro $c rc=$rc"; cat gpurun_out/repro_$c.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 5 120 python -u tools/torch_unjoined_capture.py external > gpurun_out/r4d_torch_external.log 2>&1
rc=$?; echo "torch external rc=$rc"; tail -30 gpurun_out/r4d_torch_external.log; [ $rc -eq 0 ] || exit $rc
MALLOC_PERTURB_=165 timeout -k 5 60 tools/hip_capture_repro external_event_destroyed > gpurun_out/repro_external_event_destroyed.log 2>&1
rc=$?; echo "repro external_event_destroyed rc=$rc"; cat gpurun_out/repro_external_event_destroyed.log; exit $rc
