# A/B of GEMM shapes (tools/gemm_bench.py, production dispatch) between the tree's library and an alt
# build (clipmi/alt/libclipmi_$1.so), A B A B
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
ALT=$R/vlm-clip_amd/clipmi/alt/libclipmi_$1.so; shift
export GEMM_VARIANTS=0 GEMM_REPS=${GEMM_REPS:-20}
for r in A B A B; do
  echo "== $r"
  if [ $r = A ]; then timeout -k 10 150 python3 tools/gemm_bench.py "$@"; else CLIPMI_LIB=$ALT timeout -k 10 150 python3 tools/gemm_bench.py "$@"; fi
done
