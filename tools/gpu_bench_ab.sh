#!/bin/bash
# Whole-step A/B: the train section of bench.py under each env variant given as NAME:VAR=V,...
# (e.g. base: dat0:KDPC_PC_DAT_WS=0).  Every run has its own time limit; a failure stops.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-ab}
for v in "$@"; do
  name=${v%%:*}
  envs=${v#*:}
  ( IFS=,; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done; IFS=" "
    timeout -k 10 300 python -u bench.py --sections ${SECTIONS:-train} ${BENCH_EXTRA:-} --no-cpu-baseline \
        --steps ${STEPS:-20} --warmup 3 > gpurun_out/bab_${TAG}_$name.log 2>&1 ) \
    || { echo "STOP $name"; tail -5 gpurun_out/bab_${TAG}_$name.log; exit 1; }
  python - "$name" "gpurun_out/bab_${TAG}_$name.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(f"{sys.argv[1]:10s} {d['ms_per_step']:8.3f} ms/step  {d['value']:8.2f} pairs/s  "
      f"bwd {r.get('avg_launch_us')} us frac {r.get('frac')}")
PY
done
