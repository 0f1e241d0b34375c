#!/bin/bash
# PointConv backward experiment round: parity tests of the default build, then the flow0
# microbench and the data kernel's phase stamps for the default build and each variant
# named on the command line (tools/variants/<name>, built by tools/build_variants.sh).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-exp}
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_gpu_fused.py ${EXTRA_TESTS:-} > gpurun_out/${TAG}_tests.txt 2>&1
  rc=$?; tail -2 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || { echo "STOP tests $rc"; exit $rc; }
fi
timeout -k 10 200 python tools/bench_pointconv.py ${ONLY:+--only $ONLY} > gpurun_out/${TAG}_pcb_default.txt 2>&1 || { echo STOP; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_pcb_default.txt
for v in "$@"; do
  echo "== $v"
  if [ -f tools/variants/$v/libkdpc_hip.so ]; then
    case $v in
      stamps*) KDPC_LIB=tools/variants/$v/libkdpc_hip.so timeout -k 10 200 python tools/pc_stamps.py --json gpurun_out/${TAG}_$v.json > gpurun_out/${TAG}_$v.txt 2>&1 || { echo STOP; exit 1; }
               python - "$R/gpurun_out/${TAG}_$v.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("chunk", round(d["chunk_cycles_mean"]), "prologue", round(d["prologue_share"], 3),
      {k: [round(x) for x in v] for k, v in d["phase_cycles_by_wave"].items()})
PY
               ;;
      *) KDPC_LIB=tools/variants/$v/libkdpc_hip.so timeout -k 10 200 python tools/bench_pointconv.py ${ONLY:+--only $ONLY} > gpurun_out/${TAG}_pcb_$v.txt 2>&1 || { echo STOP; exit 1; }
         grep -v amdgpu.ids gpurun_out/${TAG}_pcb_$v.txt ;;
    esac
  fi
done
echo "== done"
