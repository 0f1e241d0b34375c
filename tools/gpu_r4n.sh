#!/bin/bash
# Cross-check rerun: kernel traces of the train / kd / knn / gather sections with the
# measurement-window markers and graph-replayed microbenchmarks.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"; TAG=${1:-r04c}
for sec in ${SECS:-train kd knn gather_c3 gather_c64 configs1}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_${TAG}_$sec" -o run --output-format csv -- python3 "$R/bench.py" --sections $sec --steps 5 --warmup 2 --no-cpu-baseline > $O/kt_${TAG}_$sec.log 2>&1 || { echo "STOP kt $sec"; tail -5 $O/kt_${TAG}_$sec.log; exit 1; }
  python3 tools/roofline_check.py "$O/kt_${TAG}_$sec" $O/kt_${TAG}_$sec.log > $O/roofline_check_${TAG}_$sec.json 2>&1
  python3 -c "import json; d=json.load(open('$O/roofline_check_${TAG}_$sec.json')); print('$sec', {k: (v['rocprof_avg_us_per_launch'], v['live_hip_event_avg_us'], v['ratio_live_over_rocprof']) for k, v in d.items()})"
done
timeout -k 10 300 python -u bench.py --sections configs1,knn --no-cpu-baseline > $O/bench_${TAG}_micro.log 2>&1 || { echo "STOP micro"; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_${TAG}_micro.log') if l.startswith('{')][-1]); c=d.get('configs1', d); print({k: (v.get('avg_launch_us'), v.get('frac')) for k, v in c.items() if isinstance(v, dict) and 'frac' in v}); print('knn', d.get('roofline_knn', {}).get('avg_launch_us'))"
echo "== done"
