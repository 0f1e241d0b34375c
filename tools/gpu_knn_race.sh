#!/bin/bash
# tools/knn_race.py variants, one process each, own time limit; stop at the first failure
export TMPDIR=/tmp
mkdir -p gpurun_out/race
IFS=';' read -ra SPECS <<< "${KNN_RUNS:-main=knn}"
for spec in "${SPECS[@]}"; do
  read -ra A <<< "$spec"
  name=knn_$(echo "${A[*]}" | tr ' =' '__')
  timeout -k 10 180 python3 -u tools/knn_race.py "${A[@]}" > gpurun_out/race/$name.txt 2>&1
  rc=$?; echo "== ${A[*]} rc=$rc"; grep RESULT gpurun_out/race/$name.txt
  [ $rc -eq 0 ] || { echo "STOP $rc"; grep -v "^frame" gpurun_out/race/$name.txt | tail -8; exit $rc; }
done
