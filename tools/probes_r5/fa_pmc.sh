# PMC pass over the flash forward (attn_bench.py vision_l14_336): where a wave's cycles go
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
C="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex attn_fwd_fa --output-format csv -d $R/gpurun_out/fa_pmc -o pmc -- python3 $R/tools/attn_bench.py vision_l14_336 > $R/gpurun_out/fa_pmc.log 2>&1
