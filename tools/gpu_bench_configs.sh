#!/bin/bash
# Bench lines for the other single-GPU configs of BASELINE.json (config 2: B/32 + adapters B=256;
# config 4's model: L/14 adapter fine-tune at B=1024 per GPU) + a rocprofv3 kernel trace of the
# L/14 step.  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model B/32 --mode adapter --batch 256 --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/bench_b32_adapter.log 2>&1 || { echo "b32 bench failed rc=$?"; exit 1; }
timeout -k 10 400 python bench.py --model L/14 --mode adapter --batch 1024 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/bench_l14_adapter.log 2>&1 || { echo "l14 bench failed rc=$?"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_l14" -o l14 -- python3 "$R/bench.py" --model L/14 --mode adapter --batch 1024 --steps 3 --warmup 1 --cpu-sample 0 > "$R/gpurun_out/prof_l14.log" 2>&1 || { echo "rocprof failed rc=$?"; exit 1; }
echo all-ok
