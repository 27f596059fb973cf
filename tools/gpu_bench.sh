#!/bin/bash
# bench smoke -> full bench -> rocprofv3 kernel trace; stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --batch 64 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_small.log 2>&1 || { echo "small bench failed rc=$?"; exit 1; }
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.log 2>&1 || { echo "bench failed rc=$?"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o b16 -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-sample 0 "$@" > "$R/gpurun_out/prof.log" 2>&1 || { echo "rocprof failed rc=$?"; exit 1; }
echo all-ok
