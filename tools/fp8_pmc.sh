#!/bin/bash
# One rocprofv3 --pmc pass (MFMA busy / waits) over tools/fp8_bench.py: the MXFP8 GEMMs at L/14@336
# B = 512 (qkv, fc1, fc1_q8, fc2), FP8_VARIANTS as tools/fp8_bench.py (0 production, 40 8-wave, 41 4-wave).
# Usage: tools/fp8_pmc.sh TAG   (summary: tools/pmc_summary.py on the counter_collection.csv)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
T=${1:-f8pmc}
export FP8_REPS=1 FP8_SHAPES=${FP8_SHAPES:-qkv,fc1,fc1_q8,fc2} FP8_VARIANTS=${FP8_VARIANTS:-0,40,41}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/${T}" -o pmc -- \
  python3 "$R/tools/fp8_bench.py" > "$R/gpurun_out/${T}.log" 2>&1 || { echo "pmc pass failed rc=$?"; tail -5 "$R/gpurun_out/${T}.log"; exit 1; }
S=$(find "$R/gpurun_out/${T}" -name '*counter_collection.csv' | head -1)
python3 "$R/tools/pmc_summary.py" "$S" > "$R/gpurun_out/${T}_summary.txt"
echo all-ok
