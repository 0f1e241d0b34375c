#!/bin/bash
# Run one GPU test selection (-k $K) in each prebuilt worktree under tools/variants/ (the
# commits named on the command line); a fault / timeout stops the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
for c in "$@"; do
  cd "$R/tools/variants/$c" || exit 1
  timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
      -k "${K}" > "$R/gpurun_out/bisect_$c.log" 2>&1
  rc=$?
  echo "$c rc=$rc: $(tail -1 $R/gpurun_out/bisect_$c.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
