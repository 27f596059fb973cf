set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export GEMM_VARIANTS=0 GEMM_REPS=20
for r in A B A B; do
  if [ $r = A ]; then unset CLIPMI_RASTER; else export CLIPMI_RASTER=0; fi
  echo "== $r raster=${CLIPMI_RASTER:-auto}"
  timeout -k 10 120 python3 tools/gemm_bench.py fc1_wgrad fc2_wgrad qkv_wgrad out_wgrad t_fc2_wgrad t_fc1_wgrad
done > gpurun_out/w1_bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
export GEMM_REPS=1
for r in A B; do
  if [ $r = A ]; then unset CLIPMI_RASTER; else export CLIPMI_RASTER=0; fi
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/w1_f$r -o pmc -- python3 $R/tools/gemm_bench.py fc1_wgrad fc2_wgrad qkv_wgrad out_wgrad > $R/gpurun_out/w1_f$r.log 2>&1
  S=$(find $R/gpurun_out/w1_f$r -name '*counter_collection.csv' | head -1)
  echo "== fetch $r"; python3 $R/tools/pmc_summary.py "$S"
done > $R/gpurun_out/w1_fetch.log 2>&1
echo ok
