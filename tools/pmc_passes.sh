#!/bin/bash
# PMC passes (one rocprofv3 run per pass) over a python command; passes separated by ';' in
# $PASSES.  Usage: PASSES="A B;C D" OUT=name tools/pmc_passes.sh <python script> [args...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
OUT=${OUT:-pmc}
mkdir -p gpurun_out/$OUT
IFS=';' read -ra PS <<< "$PASSES"
i=0
for P in "${PS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "${KREGEX:-.}" -d "$R/gpurun_out/$OUT/p$i" -o run --output-format csv -- python3 "$@" > gpurun_out/$OUT/p$i.log 2>&1 || { echo "STOP pass $i"; exit 1; }
done
echo done
