# dynamic item queue for the persistent 4-wave GEMM (CLIPMI_W4P_DYN=1): GEMM + model tests with it on, bench A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CLIPMI_W4P_DYN=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/r03_dyn_test.log 2>&1
rc=$?; tail -n 1 gpurun_out/r03_dyn_test.log; grep -E "^E |FAILED" gpurun_out/r03_dyn_test.log | head -5
[ $rc -ne 0 ] && exit $rc
CLIPMI_W4P_DYN=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_model.py -k "bitwise or replay or b16" -p no:cacheprovider > gpurun_out/r03_dyn_model.log 2>&1
rc=$?; tail -n 1 gpurun_out/r03_dyn_model.log; grep -E "^E |FAILED" gpurun_out/r03_dyn_model.log | head -5
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for v in 0 1; do
  CLIPMI_W4P_DYN=$v timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/r03_dyn_$v.json 2> gpurun_out/r03_dyn_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/r03_dyn_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03_dyn_$v.json')); print('w4p_dyn $v rep $rep', d['value'], d['ms_per_step'])"
done
done
