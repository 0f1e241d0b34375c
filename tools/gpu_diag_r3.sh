#!/bin/bash
# Round-3 diagnostic pass: wide cost-volume gradient A/B vs float64, fused-vs-unfused wide
# check, then the whole-step A/B of the PointConv backward kernel variants.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/grad_ab.py > gpurun_out/grad_ab.log 2>&1 || { echo "STOP grad_ab"; tail -20 gpurun_out/grad_ab.log; exit 1; }
tail -20 gpurun_out/grad_ab.log
timeout -k 10 200 python -u tools/cv_wide_check.py > gpurun_out/cv_wide_check.log 2>&1 || { echo "STOP cvw"; tail -20 gpurun_out/cv_wide_check.log; exit 1; }
grep -v amdgpu.ids gpurun_out/cv_wide_check.log
TAG=r3a bash tools/gpu_bench_ab.sh base: dat0:KDPC_PC_DAT_WS=0 wgt0:KDPC_PC_WGT_WS=0 both0:KDPC_PC_DAT_WS=0,KDPC_PC_WGT_WS=0
