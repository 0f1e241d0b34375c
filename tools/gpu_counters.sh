#!/bin/bash
# Limiter counters of the step's MFMA kernels: one rocprofv3 --pmc pass per counter group over
# one bench section (default: train), then tools/pmc_limiters.py.  Counters the box's
# rocprofv3 -L does not list are dropped from their pass (and named in the log).
#   OUT=<name under gpurun_out> SECTION=train KREGEX=<kernel regex> tools/gpu_counters.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
OUT=${OUT:-counters}
SECTION=${SECTION:-train}
KREGEX=${KREGEX:-pc_bwd|pc_fwd|cost_volume_|cvw_fused|cv_rows_sum}
O="$R/gpurun_out/$OUT"
mkdir -p "$O"
timeout -s KILL 60 rocprofv3 -L > "$O/counters_list.txt" 2>&1 || true
CMD="python3 $R/bench.py --sections $SECTION --steps 2 --warmup 1 --no-cpu-baseline --measure-steps 1"
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
  "SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VMEM TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for P in "${PASSES[@]}"; do
  i=$((i+1))
  C=""
  for c in $P; do
    if grep -qw "${c%_sum}" "$O/counters_list.txt"; then C="$C $c"; else echo "pass $i: no counter $c"; fi
  done
  echo "pass $i:$C"
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "$KREGEX" -d "$O/p$i" -o run \
    --output-format csv -- $CMD > "$O/p$i.log" 2>&1 || { echo "STOP pass $i"; tail -5 "$O/p$i.log"; exit 1; }
done
python3 tools/pmc_limiters.py "$O" --out "$O/limiters.json" > "$O/limiters.txt" && cat "$O/limiters.txt"
echo "== done"
