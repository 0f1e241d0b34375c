#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass) over the fused PointConv microbenchmark.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/pc_pmc
export TMPDIR=/tmp
ONLY=${ONLY:-flow0}
timeout -s KILL 120 rocprofv3 -L > gpurun_out/pc_pmc/counters_list.txt 2>&1 || true
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "pc_" -d "$R/gpurun_out/pc_pmc/p$i" -o run --output-format csv -- python3 "$R/tools/bench_pointconv.py" --only "$ONLY" --iters 3 > gpurun_out/pc_pmc/p$i.log 2>&1 || { echo "STOP pass $i"; exit 1; }
done
echo done
