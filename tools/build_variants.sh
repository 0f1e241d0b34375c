#!/bin/bash
# Diagnostic builds of libkdpc_hip.so with -D flags (e.g. KDPC_WGT_MODE=1..5) into
# tools/variants/<name>/ (with a copy of the torch op library; use KDPC_LIB=<dir>/libkdpc_hip.so).
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  d=$R/tools/variants/$name; mkdir -p $d
  objs=""
  for f in $R/kd-pointcloud_amd/csrc/*.hip; do
    o=$d/$(basename $f).o
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fvisibility=hidden -Wno-unused-result -I $R/include -I $R/kd-pointcloud_amd/csrc $flags -c $f -o $o &
    objs="$objs $o"
  done
  wait
  cp $R/kd-pointcloud_amd/build/kdpc_build_id.cpp.*.o $d/id.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o $d/libkdpc_hip.so $objs $d/id.o
  cp $R/kd-pointcloud_amd/lib/libkdpc_torch.so $d/
  rm -f $d/*.o
  echo built $d
done
