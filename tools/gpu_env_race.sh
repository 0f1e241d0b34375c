#!/bin/bash
# A race tool under HIP runtime knobs: ENV_RUNS = ';'-separated "NAME=VALUE ... [-- tool args]"
# ("-" = no knob); TOOL = tools/fwd_race.py (default, args "tt") or tools/knn_race.py;
# one process each under its own limit; stop at the first failure
export TMPDIR=/tmp
mkdir -p gpurun_out/race
TOOL=${TOOL:-tools/fwd_race.py}
DEFARGS=${DEFARGS:-tt}
IFS=';' read -ra SPECS <<< "${ENV_RUNS:--}"
for spec in "${SPECS[@]}"; do
  name=env_$(basename $TOOL .py)_$(echo "$spec" | tr ' =/' '___' | cut -c1-120)
  envpart=${spec%%--*}; args=$DEFARGS; [[ "$spec" == *--* ]] && args=${spec#*--}
  envs=(); [ "$(echo $envpart)" != "-" ] && read -ra envs <<< "$envpart"
  env "${envs[@]}" timeout -k 10 200 python3 -u $TOOL $args reps=${REPS:-300} > gpurun_out/race/$name.txt 2>&1
  rc=$?; echo "== $spec rc=$rc"; grep "RESULT\|replay ms\|twice" gpurun_out/race/$name.txt
  [ $rc -eq 0 ] || { echo "STOP $rc"; grep -v "^frame" gpurun_out/race/$name.txt | tail -6; exit $rc; }
done
