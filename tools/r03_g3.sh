set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_model.py -k "b16_feature or b16_full_finetune_gradients_fp32 or trainer" > gpurun_out/r03_g3_test.log 2>&1 || { grep -E "worst|largest|Error|assert" gpurun_out/r03_g3_test.log | head; tail -5 gpurun_out/r03_g3_test.log; exit 1; }
grep -E "largest|passed|failed" gpurun_out/r03_g3_test.log
