set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k attention > gpurun_out/r03_sp2_test.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r03_sp2_test.log | head; tail -3 gpurun_out/r03_sp2_test.log; exit 1; }
tail -n 1 gpurun_out/r03_sp2_test.log
ATTN_NWS=8 ATTN_BWD_SP=1,0 timeout -k 10 200 python tools/attn_bench.py vision_b16 > gpurun_out/r03_sp2_attn.log 2>&1 || { tail -20 gpurun_out/r03_sp2_attn.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03_sp2_attn.log
