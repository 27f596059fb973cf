set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_kernels.py > gpurun_out/r03r7_test.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r03r7_test.log | head; tail -5 gpurun_out/r03r7_test.log; exit 1; }
tail -n 1 gpurun_out/r03r7_test.log
timeout -k 10 600 python bench.py > gpurun_out/r03r7_bench.json 2> gpurun_out/r03r7_bench.err || { echo "bench failed"; tail -20 gpurun_out/r03r7_bench.err; exit 1; }
cat gpurun_out/r03r7_bench.json
TAG=r03r7 bash tools/r03_prof.sh
