set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k attention > gpurun_out/r03_pad_test.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r03_pad_test.log | head; tail -3 gpurun_out/r03_pad_test.log; exit 1; }
tail -n 1 gpurun_out/r03_pad_test.log
ATTN_NWS=8 timeout -k 10 200 python tools/attn_bench.py vision_b16 text > gpurun_out/r03_pad_attn.log 2>&1 || { tail -20 gpurun_out/r03_pad_attn.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03_pad_attn.log
for rep in 1 2; do
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/r03_pad_bench.json 2> gpurun_out/r03_pad_bench.err || { echo "bench failed"; tail -5 gpurun_out/r03_pad_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r03_pad_bench.json')); print('bench', d['value'], d['ms_per_step'], d['rooflines']['attention']['avg_launch_ms'])"
done
