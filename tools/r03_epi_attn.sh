# pipelined GEMM epilogue A/B + single-pass attention backward: tests and A/B timings
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_kernels.py > gpurun_out/r03_ea_test.log 2>&1 || { tail -30 gpurun_out/r03_ea_test.log; exit 1; }
tail -n 2 gpurun_out/r03_ea_test.log
ATTN_NWS=8 ATTN_BWD_SP=1,0 timeout -k 10 200 python tools/attn_bench.py vision_b16 text > gpurun_out/r03_ea_attn.log 2>&1 || { tail -20 gpurun_out/r03_ea_attn.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03_ea_attn.log
W4_ST_PROD_ONLY=1 timeout -k 10 300 python tools/w4_stamps.py qkv_fwd_60 qkv_fwd fc1_fwd_60 fc1_fwd > gpurun_out/r03_epi_stamps.log 2>&1 || { tail -30 gpurun_out/r03_epi_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03_epi_stamps.log
SH="fc1_fwd fc2_fwd qkv_fwd out_fwd fc2_dgrad fc1_dgrad qkv_dgrad out_dgrad t_fc1_fwd t_fc2_fwd t_qkv_fwd t_fc2_dgrad"
GEMM_VARIANTS=0,28 timeout -k 10 400 python tools/gemm_bench.py $SH > gpurun_out/r03_epi_new.log 2>&1
CLIPMI_LIB=$GRAFT_REPO_ROOT/vlm-clip_amd/alt/libclipmi_old_epi.so GEMM_VARIANTS=0,28 timeout -k 10 400 python tools/gemm_bench.py $SH > gpurun_out/r03_epi_old.log 2>&1
echo "== new"; grep -v amdgpu.ids gpurun_out/r03_epi_new.log
echo "== old"; grep -v amdgpu.ids gpurun_out/r03_epi_old.log
timeout -k 10 600 python bench.py > gpurun_out/r03_ea_bench.json 2> gpurun_out/r03_ea_bench.err || { echo "bench failed"; tail -20 gpurun_out/r03_ea_bench.err; exit 1; }
cat gpurun_out/r03_ea_bench.json
