#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q --timeout 200 --timeout-method thread -k "batchnorm" > gpurun_out/r4g_bn.log 2>&1 || { tail -20 gpurun_out/r4g_bn.log; exit 1; }
tail -1 gpurun_out/r4g_bn.log
timeout -k 10 300 python -u tools/entry_rooflines.py --json gpurun_out/entry_rooflines_r04.json > gpurun_out/r4g_entry.log 2>&1
rc=$?; tail -30 gpurun_out/r4g_entry.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
TAG=cvp bash tools/gpu_bench_ab.sh base: plain:KDPC_CV_BWD_PLAIN=1 base2: plain2:KDPC_CV_BWD_PLAIN=1
grep -h host_issue gpurun_out/bab_cvp_base.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('host issue ms/step', d.get('host_issue_ms_per_step'), 'enqueue', d.get('host_enqueue_ms'))"
timeout -k 10 300 python -u tools/torch_profile.py --out gpurun_out/torch_prof_r04.txt > gpurun_out/r4g_tprof.log 2>&1
rc=$?; echo "torch profile rc=$rc"
