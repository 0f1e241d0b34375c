#!/bin/bash
# Round-6 measurement of the committed tree: the default bench line, rocprofv3 kernel traces
# of the train and KD sections (cross-check of the live rooflines: tools/roofline_check.py),
# and one FETCH_SIZE and one WRITE_SIZE pass per section for the HBM traffic
# (tools/pmc_traffic.py merges them on the CPU side).  Every GPU step under its own limit;
# the first failure stops the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 600 python3 bench.py > $O/bench.txt 2>&1 || { echo "STOP bench"; tail -5 $O/bench.txt; exit 1; }
tail -1 $O/bench.txt | cut -c1-300
KREGEX="pc_|group_rows|group_points|cost_volume_|cvw_|cv_rows|idw_|csr_|colsum"
for sec in train kd; do
  CMD="python3 $R/bench.py --sections $sec --steps 3 --warmup 2 --no-cpu-baseline"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/$O/kt_$sec" -o run --output-format csv -- $CMD > $O/kt_$sec.log 2>&1 || { echo "STOP kt $sec"; tail -5 $O/kt_$sec.log; exit 1; }
  grep -E '"metric"|^\{"kd_step"' $O/kt_$sec.log > $O/kt_bench_$sec.json || true
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KREGEX" -d "$R/$O/pmcf_$sec" -o run --output-format csv -- $CMD > $O/pmcf_$sec.log 2>&1 || { echo "STOP pmc fetch $sec"; tail -5 $O/pmcf_$sec.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KREGEX" -d "$R/$O/pmcw_$sec" -o run --output-format csv -- $CMD > $O/pmcw_$sec.log 2>&1 || { echo "STOP pmc write $sec"; tail -5 $O/pmcw_$sec.log; exit 1; }
  echo "== $sec done"
done
echo "== done"
