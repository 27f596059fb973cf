# round-3 end: full GPU suite + bench + rocprof kernel stats of the bench + roofline cross-check
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r03fin bash tools/r03_full.sh || exit 1
TAG=r03fin bash tools/r03_prof.sh || exit 1
