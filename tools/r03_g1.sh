set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
GEMM_TORCH=1 GEMM_VARIANTS=0,12 timeout -k 10 300 python tools/gemm_bench.py fc1_fwd fc2_fwd qkv_fwd out_fwd fc2_dgrad fc1_wgrad sq8k > gpurun_out/r03_g1_gemm.log 2>&1
cat gpurun_out/r03_g1_gemm.log | grep -v amdgpu.ids
GEMM_TORCH=1 GEMM_VARIANTS=0 GEMM_REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_g1_prof -o g -- python3 tools/gemm_bench.py fc1_fwd fc2_fwd qkv_fwd fc2_dgrad fc1_wgrad sq8k > gpurun_out/r03_g1_prof.log 2>&1
S=$(find gpurun_out/r03_g1_prof -name '*kernel_stats.csv' | head -1)
cut -c1-400 $S | head -30
