#!/bin/bash
# Round 6 perf: KD step with the teacher as a branch of one graph vs a graph of its own, and
# the per-kernel table of the train and KD steps (rocprofv3 kernel trace).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r6
TAG=${TAG:-p1}
for tg in 0 1; do
  KDPC_TEACHER_GRAPH=$tg timeout -k 10 300 python3 bench.py --sections kd --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r6/kd_tg${tg}_$TAG.txt 2>&1 || { echo "STOP kd $tg"; tail -5 gpurun_out/r6/kd_tg${tg}_$TAG.txt; exit 1; }
  python3 -c "import json,sys; l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d=json.loads(l); k=d.get('kd_step',d); print('teacher_graph=$tg', k['value'], k['ms_per_step'], k.get('step'))" gpurun_out/r6/kd_tg${tg}_$TAG.txt
done
for sec in train kd; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r6/kt_${sec}_$TAG" -o run --output-format csv -- python3 "$R/bench.py" --sections $sec --steps 4 --warmup 2 --no-cpu-baseline --measure-steps 0 > gpurun_out/r6/kt_${sec}_$TAG.log 2>&1 || { echo "STOP kt $sec"; tail -5 gpurun_out/r6/kt_${sec}_$TAG.log; exit 1; }
done
echo "== done"
