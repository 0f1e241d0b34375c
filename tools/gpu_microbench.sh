set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/microbench_ops.py --json gpurun_out/microbench.json > gpurun_out/mb.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mbprof -o run --output-format csv -- python3 tools/microbench_ops.py > gpurun_out/mbprof.log 2>&1 || exit $?
echo done
