set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/r03_st2.sh
TAG=r03s2 bash tools/r03_full.sh
