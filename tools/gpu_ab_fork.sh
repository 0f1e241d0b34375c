#!/bin/bash
# A/B of the decoder coordinate fork (KDPC_COORD_FORK) on the train and KD steps, interleaved.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
true
TAG=fkkd STEPS=30 SECTIONS=kd BENCH_EXTRA="--mode kd --batch 4" bash tools/gpu_bench_ab.sh off:KDPC_COORD_FORK=0 on:KDPC_COORD_FORK=1 off2:KDPC_COORD_FORK=0 on2:KDPC_COORD_FORK=1
