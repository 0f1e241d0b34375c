#!/bin/bash
# Split-K geometry of the dense weight gradients: train/KD A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
for rnd in 1 2; do
  for v in ${VALS:-1024,128 512,256 1024,256 512,128 256,512}; do
    KDPC_SPLITK=$v timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/r4y_b.log 2>&1 || { echo "STOP b $v"; tail -5 $O/r4y_b.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/r4y_b.log') if l.startswith('{')][-1]); print('splitk=$v', d['ms_per_step'], d['kd_step']['ms_per_step'])"
  done
done
echo "== done"
