#!/bin/bash
# Side-stream weight-kernel CU budget A/B (KDPC_PC_WGT_CUS): train + KD step times.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
for rnd in 1 2; do
  for w in ${CUS:-256 192 128 64}; do
    KDPC_PC_WGT_CUS=$w timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/r4r_${w}_$rnd.log 2>&1 || { echo "STOP $w"; tail -5 $O/r4r_${w}_$rnd.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/r4r_${w}_$rnd.log') if l.startswith('{')][-1]); print('cus=$w', d['ms_per_step'], d['kd_step']['ms_per_step'])"
  done
done
echo "== done"
