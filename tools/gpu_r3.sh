#!/bin/bash
# Round-3 GPU pass: GPU tests (all, or the -k expression in $K), then the default bench line.
# A test failure (pytest rc 1) still runs the bench; a fault / abort / timeout (any other rc)
# stops the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-a}
SEL=()
if [ -n "${K:-}" ]; then SEL=(-k "$K"); fi
timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest tests -m gpu -v --timeout 300 \
    --timeout-method thread ${PYARGS:-} "${SEL[@]}" > gpurun_out/r3_pytest_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/r3_pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP pytest rc=$rc"; exit $rc; fi
if [ -n "${NOBENCH:-}" ]; then exit $rc; fi
timeout -k 10 ${BENCH_LIMIT:-500} python -u bench.py ${BENCH_ARGS:-} > gpurun_out/r3_bench_$TAG.log 2>&1
brc=$?
tail -2 gpurun_out/r3_bench_$TAG.log
echo "pytest rc=$rc bench rc=$brc"
exit $brc
