# bias prefetch: GEMM tests + shapes, then the two-stream CU-sharing A/B (grid cap, serial towers)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/r03r10_test.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r03r10_test.log | head; tail -5 gpurun_out/r03r10_test.log; exit 1; }
tail -n 1 gpurun_out/r03r10_test.log
GEMM_VARIANTS=0,28 timeout -k 10 400 python tools/gemm_bench.py qkv_fwd out_fwd fc1_fwd_dact fc2_fwd t_qkv_fwd t_fc1_fwd_dact > gpurun_out/r03r10_gemm.log 2>&1
grep -v amdgpu.ids gpurun_out/r03r10_gemm.log
bash tools/r03_run9.sh
