#!/bin/bash
# Counter profile of the D<=64 cost-volume backward kernel (tools/bench_cv_bwd.py shapes)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$R/gpurun_out"
P1="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS,SQ_INSTS_VALU"
P2="SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_BUSY_CYCLES,SQ_WAVES,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR"
i=1
for P in $P1 $P2; do
  timeout -s KILL 120 rocprofv3 --pmc ${P//,/ } --kernel-include-regex "cost_volume_bwd_kernel|pc_bwd_data" -d "$O/cvpmc_$i" -o run --output-format csv -- python3 "$R/tools/bench_cv_bwd.py" --iters 3 > $O/cvpmc_$i.log 2>&1 || { echo "STOP pass $i"; tail -5 $O/cvpmc_$i.log; exit 1; }
  echo "pass $i ok"; i=$((i+1))
done
