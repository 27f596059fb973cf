cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03p}
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o b16 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --cpu-sample 0 > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log 2>&1 || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
S=$(find gpurun_out/${T}_prof -name '*kernel_trace.csv' | head -1)
python3 tools/stream_breakdown.py $S 4
python3 tools/roofline_check.py $S
