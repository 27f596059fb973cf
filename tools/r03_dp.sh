cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_dp.py -v -x --timeout 240 --timeout-method thread -p no:cacheprovider 2>&1 | tee gpurun_out/r03_dp.log
