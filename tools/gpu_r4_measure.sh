#!/bin/bash
# Round-4 measurement pass.  Step 1: the default bench line.  Step 2: per-section rocprofv3
# kernel traces (live roofline vs rocprof cross-check).  Step 3: PMC FETCH_SIZE / WRITE_SIZE
# passes per workload (separate runs, MI355X_MICROARCH.md §HBM).
# Every GPU step has its own time limit; any failure ends the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04}
PARTS=${PARTS:-bench,kt,pmc}
SECS=${SECS:-train kd configs1 knn gather_c3 gather_c64}
O="$R/gpurun_out"
if [[ $PARTS == *bench* ]]; then
  timeout -k 10 500 python -u bench.py > $O/bench_$TAG.log 2>&1 || { echo "STOP bench"; tail -5 $O/bench_$TAG.log; exit 1; }
  tail -1 $O/bench_$TAG.log | cut -c1-400
fi
if [[ $PARTS == *kt* ]]; then
  for sec in $SECS; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_${TAG}_$sec" -o run --output-format csv -- python3 "$R/bench.py" --sections $sec --steps 5 --warmup 2 --no-cpu-baseline > $O/kt_${TAG}_$sec.log 2>&1 || { echo "STOP kt $sec"; tail -5 $O/kt_${TAG}_$sec.log; exit 1; }
    python3 tools/roofline_check.py "$O/kt_${TAG}_$sec" $O/kt_${TAG}_$sec.log > $O/roofline_check_${TAG}_$sec.json 2>&1
    echo "kt $sec ok: $(tr -d '\n ' < $O/roofline_check_${TAG}_$sec.json | cut -c1-300)"
  done
fi
if [[ $PARTS == *pmc* ]]; then
  RE="pc_|group_rows|group_points|gather_points|cost_volume_|cvw_|cv_rows|idw_|knn|ref_sort|query_sort|chunk_box"
  for sec in $SECS; do
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "$RE" -d "$O/pmc_${TAG}_${sec}_$c" -o run --output-format csv -- python3 "$R/bench.py" --sections $sec --steps 2 --warmup 1 --no-cpu-baseline --measure-steps 1 > $O/pmc_${TAG}_${sec}_$c.log 2>&1 || { echo "STOP pmc $sec $c"; tail -5 $O/pmc_${TAG}_${sec}_$c.log; exit 1; }
    done
    echo "pmc $sec ok"
  done
fi
echo "== done"
