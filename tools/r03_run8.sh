# config 5 bench line, fp8 GEMM shapes, PMC passes of the production MXFP8 kernel, wgrad traffic
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --model L/14@336 --mode adapter --precision fp8 --batch 4096 --steps 4 --warmup 2 --cpu-sample 0 > gpurun_out/r03r8_cfg5.json 2> gpurun_out/r03r8_cfg5.err || { echo "cfg5 bench failed"; tail -20 gpurun_out/r03r8_cfg5.err; exit 1; }
cat gpurun_out/r03r8_cfg5.json
timeout -k 10 300 python tools/fp8_bench.py 512 > gpurun_out/r03r8_fp8.log 2>&1 || { tail -20 gpurun_out/r03r8_fp8.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03r8_fp8.log
cd /tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE TA_BUSY_avr TA_BUSY_max"; do
  i=$((i + 1))
  FP8_REPS=1 FP8_SHAPES=qkv,fc1,fc2 timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/r03r8_fp8pmc_p$i" -o pmc -- \
    python3 "$R/tools/fp8_bench.py" 512 > "$R/gpurun_out/r03r8_fp8pmc_p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$R/gpurun_out/r03r8_fp8pmc_p$i.log"; exit 1; }
done
cd $R
for j in 1 2; do
  S=$(find gpurun_out/r03r8_fp8pmc_p$j -name '*counter_collection.csv' | head -1)
  echo "== pass $j"; python3 tools/pmc_summary.py "$S" | grep -i "fp8\|quant\|ln_fwd" | head -20
done
bash tools/traffic_pmc.sh r03r8
