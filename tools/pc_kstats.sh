#!/bin/bash
# rocprofv3 kernel stats of the PointConv microbench (ONLY=flow0 by default) for the default
# build (PIPE=0 and 1) and each tools/variants/<name> given (KDPC_PC_BWD_PIPE=${VPIPE:-0}):
# the per-kernel average durations of the pc_* kernels.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-ks}
run() {  # name, pipe, lib
  local d="$R/gpurun_out/${TAG}_$1"
  KDPC_LIB=$3 KDPC_PC_BWD_PIPE=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d" -o run --output-format csv -- python3 "$R/tools/bench_pointconv.py" --only ${ONLY:-flow0} > "$d.log" 2>&1 || { echo "STOP $1"; exit 1; }
  f=$(find "$d" -name "*kernel_stats.csv" | head -1)
  python3 "$R/tools/kstats_short.py" "$f" "$1" --filter pc_
}
DEF=$R/kd-pointcloud_amd/lib/libkdpc_hip.so
[ "${BASE:-1}" = "1" ] && { run base0 0 $DEF; run base1 1 $DEF; }
for v in "$@"; do run $v ${VPIPE:-0} $R/tools/variants/$v/libkdpc_hip.so; done
echo "== done"
