#!/bin/bash
# A/B: what part of the coordinate fork pays (kNN alone vs kNN + CSRs), train and KD steps.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
TAG=fc STEPS=30 bash tools/gpu_bench_ab.sh off:KDPC_COORD_FORK=0 knn:KDPC_COORD_FORK_CSR=0 both:KDPC_COORD_FORK_CSR=1 off2:KDPC_COORD_FORK=0 knn2:KDPC_COORD_FORK_CSR=0 both2:KDPC_COORD_FORK_CSR=1 || exit 1
TAG=fckd STEPS=30 SECTIONS=kd BENCH_EXTRA="--mode kd --batch 4" bash tools/gpu_bench_ab.sh off:KDPC_KD_COORD_FORK=0 knn:KDPC_KD_COORD_FORK=1,KDPC_COORD_FORK_CSR=0 off2:KDPC_KD_COORD_FORK=0 knn2:KDPC_KD_COORD_FORK=1,KDPC_COORD_FORK_CSR=0
