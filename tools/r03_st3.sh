# epilogue decomposition (fc1 / fc2-dgrad shapes, 4-wave stamped kernel) + single-pass attention A/B
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k attention > gpurun_out/r03_st3_test.log 2>&1 || { tail -30 gpurun_out/r03_st3_test.log; exit 1; }
tail -n 1 gpurun_out/r03_st3_test.log
ATTN_NWS=8 ATTN_BWD_SP=1,0 timeout -k 10 200 python tools/attn_bench.py vision_b16 > gpurun_out/r03_st3_attn.log 2>&1 || { tail -20 gpurun_out/r03_st3_attn.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03_st3_attn.log
W4_ST_PROD_ONLY=1 timeout -k 10 300 python tools/w4_stamps.py fc1_fwd fc1_fwd_nopre fc1_fwd_bias qkv_fwd fc2_dgrad fc2_dgrad_plain > gpurun_out/r03_st3.log 2>&1 || { tail -30 gpurun_out/r03_st3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03_st3.log
