set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/w4_stamps.py fc1_dgrad qkv_fwd > gpurun_out/r03_st.log 2>&1 || { tail -30 gpurun_out/r03_st.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03_st.log
