set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k "4wave or wgrad" > gpurun_out/r03_wg_test.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r03_wg_test.log | head -20; tail -3 gpurun_out/r03_wg_test.log; exit 1; }
tail -1 gpurun_out/r03_wg_test.log
GEMM_VARIANTS=4,28 timeout -k 10 300 python tools/gemm_bench.py fc1_wgrad fc2_wgrad qkv_wgrad out_wgrad > gpurun_out/r03_wg_gemm.log 2>&1
grep -v amdgpu.ids gpurun_out/r03_wg_gemm.log
