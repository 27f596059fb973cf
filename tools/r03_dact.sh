# stored quick_gelu' (fc1 forward) + plain product (fc2 dgrad): GPU suite parts, stamps, GEMM shapes, bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for f in tests/test_gpu_gemm.py tests/test_gpu_kernels.py tests/test_gpu_model.py; do
  n=$(basename $f .py)
  timeout -k 10 600 python -u -m pytest $f -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r03d_$n.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/r03d_$n.log | head -20; exit 1; }
  echo "$f $(tail -n 1 gpurun_out/r03d_$n.log)"
done
W4_ST_PROD_ONLY=1 timeout -k 10 300 python tools/w4_stamps.py fc1_fwd_dact fc2_dgrad_ma qkv_fwd > gpurun_out/r03d_st.log 2>&1 || { tail -30 gpurun_out/r03d_st.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03d_st.log
GEMM_VARIANTS=0,28 timeout -k 10 400 python tools/gemm_bench.py fc1_fwd fc1_fwd_dact fc2_dgrad fc2_dgrad_ma qkv_fwd out_fwd fc2_fwd t_fc1_fwd_dact t_fc2_dgrad_ma > gpurun_out/r03d_gemm.log 2>&1
grep -v amdgpu.ids gpurun_out/r03d_gemm.log
timeout -k 10 600 python bench.py > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err || { echo "bench failed"; tail -20 gpurun_out/r03d_bench.err; exit 1; }
cat gpurun_out/r03d_bench.json
