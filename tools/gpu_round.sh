#!/bin/bash
# One GPU pass: the -m gpu suite file by file (stop at the first crash), then the default bench.
# Usage: tools/gpu_round.sh TAG [test files...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
T=${1:-r}; shift
FILES=${@:-tests/test_gpu_kernels.py tests/test_gpu_gemm.py tests/test_gpu_model.py tests/test_gpu_heads.py tests/test_gpu_dp.py}
for f in $FILES; do
  name=$(basename "$f" .py)
  timeout -k 10 900 python -u -m pytest "$f" -q -p no:cacheprovider -s --timeout 300 --timeout-method thread -m gpu > "gpurun_out/${T}_$name.log" 2>&1
  rc=$?
  echo "$f rc=$rc $(tail -1 gpurun_out/${T}_$name.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after crash rc=$rc"; exit $rc; fi
done
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
  cat gpurun_out/${T}_bench.json
fi
echo all-ok
