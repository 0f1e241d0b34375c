#!/bin/bash
# Packed-math FPS: bit-exact FPS tests (incl. the model's 8192 -> 2048 chain), configs1 FPS time.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_kernels.py tests/test_gpu_kd.py -k "fps or furthest or plan" > $O/r4q_t.log 2>&1 || { echo "STOP t"; tail -30 $O/r4q_t.log; exit 1; }
tail -1 $O/r4q_t.log
timeout -k 10 300 python -u bench.py --sections configs1 --no-cpu-baseline > $O/r4q_b.log 2>&1 || { echo "STOP b"; tail -5 $O/r4q_b.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/r4q_b.log') if l.startswith('{')][-1]); c=d.get('configs1', d); print(c['fps'])"
echo "== done"
