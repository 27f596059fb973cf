#!/bin/bash
# GPU perf pass: per-shape GEMM bench -> full bench.py -> rocprofv3 kernel stats of a short
# bench run.  Stops at the first failing step.  Usage: tools/gpu_perf.sh TAG [bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
T=${1:-run}; shift
if [ -z "$SKIP_GEMM" ]; then
  timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/${T}_gemm.log 2>&1 || { echo "gemm_bench failed rc=$?"; tail -20 gpurun_out/${T}_gemm.log; exit 1; }
  cat gpurun_out/${T}_gemm.log | grep -v amdgpu.ids
fi
timeout -k 10 600 python bench.py "$@" > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${T}_prof" -o b16 -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-sample 0 "$@" > "$R/gpurun_out/${T}_prof.log" 2>&1 || { echo "rocprof failed rc=$?"; tail -20 "$R/gpurun_out/${T}_prof.log"; exit 1; }
S=$(find "$R/gpurun_out/${T}_prof" -name '*kernel_stats.csv' | head -1)
python3 "$R/tools/prof_summary.py" "$S" 4 30
echo all-ok
