cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cp in 0 1 2 3; do
  if [ $cp = 0 ]; then L=""; else L=$PWD/vlm-clip_amd/alt/libclipmi_cp$cp.so; fi
  echo "== cache policy $cp"
  CLIPMI_LIB=$L GEMM_VARIANTS=28 timeout -k 10 200 python tools/gemm_bench.py fc1_dgrad qkv_fwd fc2_fwd fc1_fwd sq8k 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r03_cp.log || exit 1
done
