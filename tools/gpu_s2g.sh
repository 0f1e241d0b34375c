#!/bin/bash
# smoke(), then the D<=64 cost-volume backward's queries-per-wave A/B in the whole step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke_s2g.log 2>&1 || { echo "STOP smoke"; tail -5 $O/smoke_s2g.log; exit 1; }
tail -1 $O/smoke_s2g.log
run() {
  env "$@" timeout -k 10 300 python -u bench.py --sections train,kd --no-cpu-baseline > $O/s2g_b.log 2>&1 || { echo "STOP $*"; tail -5 $O/s2g_b.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/s2g_b.log') if l.startswith('{')][-1]); print('$*', d['ms_per_step'], d['kd_step']['ms_per_step'])"
}
for rnd in 1 2; do
  run X=0
  run KDPC_CV_BWD_QPW=8
  run KDPC_CV_BWD_QPW=16
  run KDPC_CV_BWD_QPW=32
done
echo "== done"
