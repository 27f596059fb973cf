set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
W4_ST_PROD_ONLY=1 timeout -k 10 300 python tools/w4_stamps.py qkv_fwd_60 qkv_fwd fc1_fwd_60 fc1_fwd > gpurun_out/r03_st2.log 2>&1 || { tail -30 gpurun_out/r03_st2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03_st2.log
