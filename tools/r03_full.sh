# full GPU suite (one process per file, stop on crash), then bench + rocprof kernel stats
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03full}
for f in tests/test_gpu_gemm.py tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_heads.py tests/test_gpu_dp.py; do
  n=$(basename $f .py)
  timeout -k 10 600 python -u -m pytest $f -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_$n.log 2>&1
  rc=$?
  echo "$f rc=$rc $(tail -1 gpurun_out/${T}_$n.log)"
  if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/${T}_$n.log | head -15; exit $rc; fi
done
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
