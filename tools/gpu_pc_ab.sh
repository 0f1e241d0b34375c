#!/bin/bash
# A/B of the PointConv backward kernels (KDPC_PC_WGT_WS / KDPC_PC_DAT_WS): microbench times, bitwise
# comparison of every backward output, and a rocprofv3 kernel-trace of the flow0 shape.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ab}
if [ -n "${PRE:-}" ]; then
  timeout -k 10 300 bash -c "$PRE" > gpurun_out/pre_$TAG.log 2>&1 || { echo "STOP pre"; cat gpurun_out/pre_$TAG.log | tail -20; exit 1; }
  tail -40 gpurun_out/pre_$TAG.log
fi
# base = both single-role kernels, w = WS weight kernel, wd = WS weight + WS data kernel
for v in base:0:0 w:1:0 wd:1:1; do
  IFS=: read -r name wg da <<< "$v"
  KDPC_PC_WGT_WS=$wg KDPC_PC_DAT_WS=$da timeout -k 10 200 python -u tools/bench_pointconv.py \
      --dump /tmp/pc_$name.npz > gpurun_out/pc_${name}_$TAG.log 2>&1 || { echo "STOP $name"; tail gpurun_out/pc_${name}_$TAG.log; exit 1; }
  echo "== $name"; grep -v amdgpu.ids gpurun_out/pc_${name}_$TAG.log
done
python - <<'PY'
import numpy as np
a = np.load("/tmp/pc_base.npz")
for name in ("w", "wd"):
    b = np.load(f"/tmp/pc_{name}.npz")
    for k in a.files:
        same = np.array_equal(a[k], b[k])
        d = float(np.abs(a[k].astype(np.float64) - b[k]).max()) if not same else 0.0
        print(name, "bitwise" if same else "DIFF", k, a[k].shape, d)
PY
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kt_pc_$TAG" -o run --output-format csv -- python3 tools/bench_pointconv.py --only flow0 > gpurun_out/kt_pc_$TAG.log 2>&1 || { echo "STOP kt"; exit 1; }
f=$(find gpurun_out/kt_pc_$TAG -name "*kernel_stats.csv" | head -1)
head -12 "$f" | cut -c1-200
