set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_model.py -k "b16_feature or b16_full_finetune_gradients_fp32" > gpurun_out/r03_g2_test.log 2>&1 || { grep -E "worst|largest|Error|assert" gpurun_out/r03_g2_test.log | head; tail -5 gpurun_out/r03_g2_test.log; exit 1; }
grep -E "largest|passed|failed" gpurun_out/r03_g2_test.log
GEMM_VARIANTS=0,9 timeout -k 10 400 python tools/gemm_bench.py fc2_fwd fc1_dgrad qkv_dgrad t_fc2_fwd t_fc1_dgrad t_qkv_dgrad t_fc2_dgrad > gpurun_out/r03_g2_gemm.log 2>&1
grep -v amdgpu.ids gpurun_out/r03_g2_gemm.log
