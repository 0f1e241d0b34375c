#!/bin/bash
# KD teacher-stream race diagnostics (tools/kd_race.py); each run under its own limit.
# RACE_RUNS: ';'-separated "name mode key=value ..." entries
export TMPDIR=/tmp
mkdir -p gpurun_out/race
IFS=';' read -ra SPECS <<< "${RACE_RUNS:-gg_a gg teach=1 steps=24}"
for spec in "${SPECS[@]}"; do
  read -ra A <<< "$spec"
  name=${A[0]}
  timeout -k 10 300 python3 -u tools/kd_race.py "${A[@]:1}" > gpurun_out/race/$name.txt 2>&1
  rc=$?; echo "== $name rc=$rc"; grep -E "RESULT|CSAN errors" gpurun_out/race/$name.txt
  [ $rc -eq 0 ] || { echo "STOP $name $rc"; tail -5 gpurun_out/race/$name.txt; exit $rc; }
done
