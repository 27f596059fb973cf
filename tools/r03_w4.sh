set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k "4wave" > gpurun_out/r03_w4_test.log 2>&1 || { tail -30 gpurun_out/r03_w4_test.log; exit 1; }
tail -3 gpurun_out/r03_w4_test.log
GEMM_VARIANTS=${VARS:-0,20,28,29,30} timeout -k 10 400 python tools/gemm_bench.py ${SHAPES:-fc1_fwd fc2_fwd qkv_fwd out_fwd fc2_dgrad fc1_dgrad qkv_dgrad out_dgrad t_fc1_fwd t_qkv_fwd sq8k} > gpurun_out/r03_w4_gemm.log 2>&1
grep -v amdgpu.ids gpurun_out/r03_w4_gemm.log
