#!/bin/bash
# Run GPU steps in order; stop at the first step that crashes, aborts, times out or fails
# (pytest exit 1 = test failures -> also stop, nothing else runs on a failing tree).
# usage: tools/gpu_run.sh "<step1>" "<step2>" ...   (each step: a command line, run under bash)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
i=0
for step in "$@"; do
  i=$((i+1))
  echo "== step $i: $step"
  bash -c "$step"
  rc=$?
  if [ $rc -ne 0 ]; then echo "STOP: step $i exit $rc"; exit $rc; fi
done
echo "== all steps ok"
