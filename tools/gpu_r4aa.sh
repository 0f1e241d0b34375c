#!/bin/bash
# Side-stream geometry A/B: weight-kernel CU budget beyond one round, colsum level-1 target.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
run() {
  env "$@" timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/r4aa_b.log 2>&1 || { echo "STOP $*"; tail -5 $O/r4aa_b.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/r4aa_b.log') if l.startswith('{')][-1]); print('$*', d['ms_per_step'], d['kd_step']['ms_per_step'])"
}
for rnd in 1 2 3; do
  run KDPC_WGRAD_STREAMS=1
  run KDPC_WGRAD_STREAMS=2
  run KDPC_WGRAD_STREAMS=3
done
echo "== done"
