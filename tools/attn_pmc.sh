#!/bin/bash
# PMC passes over the attention kernels of tools/attn_bench.py (B/16, text, L/14, L/14@336 shapes):
# MFMA busy / LDS waits / bank conflicts in one pass, FETCH_SIZE and WRITE_SIZE in their own
# (MI355X_MICROARCH.md "rocprofv3 PMC slots").  Usage: tools/attn_pmc.sh TAG -> gpurun_out/TAG_attn_*
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-attn}
cd /tmp && export TMPDIR=/tmp
i=0
for C in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" FETCH_SIZE WRITE_SIZE; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex attn --output-format csv -d "$R/gpurun_out/${T}_attn_p$i" -o pmc -- \
    python3 "$R/tools/attn_bench.py" > "$R/gpurun_out/${T}_attn_p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$R/gpurun_out/${T}_attn_p$i.log"; exit 1; }
done
echo all-ok
