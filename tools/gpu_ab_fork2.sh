#!/bin/bash
# A/B: decoder coordinate fork on the parameter-gradient stream vs its own stream (train),
# and fork on/off for the KD student (shared stream).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
TAG=fs STEPS=30 bash tools/gpu_bench_ab.sh own:KDPC_COORD_OWN_STREAM=1 shared:KDPC_COORD_OWN_STREAM=0 own2:KDPC_COORD_OWN_STREAM=1 shared2:KDPC_COORD_OWN_STREAM=0 || exit 1
TAG=fskd STEPS=30 SECTIONS=kd BENCH_EXTRA="--mode kd --batch 4" bash tools/gpu_bench_ab.sh off:KDPC_KD_COORD_FORK=0 on:KDPC_KD_COORD_FORK=1 off2:KDPC_KD_COORD_FORK=0 on2:KDPC_KD_COORD_FORK=1
