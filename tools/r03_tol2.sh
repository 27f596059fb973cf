cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -s -q --timeout 240 --timeout-method thread tests/test_gpu_model.py -k "b16_full or fp8_towers or b256 or batch64" -p no:cacheprovider > gpurun_out/r03_tol2.log 2>&1
rc=$?
grep -E "^\[|passed|failed|Error|assert" gpurun_out/r03_tol2.log | head -40
exit $rc
