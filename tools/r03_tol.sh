# measured values behind the model-level tolerances (prints of the gradient / fp8 / config-2 tests)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -s -q --timeout 240 --timeout-method thread tests/test_gpu_model.py -k "gradients or fp8 or b256 or forward_matches" -p no:cacheprovider > gpurun_out/r03_tol.log 2>&1
rc=$?
grep -E "^\[|passed|failed" gpurun_out/r03_tol.log | head -80
exit $rc
