#!/bin/bash
# PMC passes over tools/gemm_bench.py for the named shapes, one rocprofv3 --pmc run per
# counter group (MI355X_MICROARCH.md "rocprofv3 PMC slots").  Usage: tools/gemm_pmc.sh TAG shape...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
T=${1:-pmc}; shift
export GEMM_VARIANTS=${GEMM_VARIANTS:-0} GEMM_REPS=${GEMM_REPS:-1}
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE TA_BUSY_avr TA_BUSY_max" \
         "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/${T}_p$i" -o pmc -- \
    python3 "$R/tools/gemm_bench.py" "$@" > "$R/gpurun_out/${T}_p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$R/gpurun_out/${T}_p$i.log"; exit 1; }
done
for j in $(seq 1 $i); do
  S=$(find "$R/gpurun_out/${T}_p$j" -name '*counter_collection.csv' | head -1)
  echo "== pass $j"; python3 "$R/tools/pmc_summary.py" "$S"
done
echo all-ok
