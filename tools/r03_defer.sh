# deferred split-K reduces (CLIPMI_DEFER_REDUCE=1): bf16 model tests with it on, then bench A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CLIPMI_DEFER_REDUCE=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_model.py -k "bf16 or replay or bitwise or trainer or b256" -p no:cacheprovider > gpurun_out/r03_defer_test.log 2>&1
rc=$?
tail -n 2 gpurun_out/r03_defer_test.log; grep -E "^E |FAILED" gpurun_out/r03_defer_test.log | head
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for v in 0 1; do
  CLIPMI_DEFER_REDUCE=$v timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/r03_defer_$v.json 2> gpurun_out/r03_defer_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/r03_defer_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03_defer_$v.json')); print('defer_reduce $v rep $rep', d['value'], d['ms_per_step'])"
done
done
