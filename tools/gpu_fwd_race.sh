#!/bin/bash
# tools/fwd_race.py variants, one process each, own time limit; stop at the first failure
export TMPDIR=/tmp
mkdir -p gpurun_out/race
IFS=';' read -ra SPECS <<< "${FWD_RUNS:-ts}"
for spec in "${SPECS[@]}"; do
  read -ra A <<< "$spec"
  name=fwd_$(echo "${A[*]}" | tr ' =' '__')
  timeout -k 10 240 python3 -u tools/fwd_race.py "${A[@]}" > gpurun_out/race/$name.txt 2>&1
  rc=$?; echo "== ${A[*]} rc=$rc"; grep RESULT gpurun_out/race/$name.txt
  [ $rc -eq 0 ] || { echo "STOP $rc"; grep -v "^frame" gpurun_out/race/$name.txt | tail -8; exit $rc; }
done
