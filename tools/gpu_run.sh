#!/bin/bash
# One parameterised GPU runner (replaces round 3's per-experiment r03_*.sh scripts).
#   tools/gpu_run.sh TAG STEP [STEP ...]
# Every step runs under its own time limit; the script stops at the first failing step and never
# retries.  Outputs go to gpurun_out/TAG_<step>.log.  Steps:
#   tests[=FILES]        pytest -m gpu (default: the whole suite, one process)
#   bench[=ARGS]         python bench.py ARGS (comma-separated args, e.g. bench=--steps,20)
#   gemm=VARIANTS:SHAPES tools/gemm_bench.py with GEMM_VARIANTS=VARIANTS on comma-separated SHAPES
#   attn[=ARGS]          tools/attn_bench.py ARGS
#   fp8[=ARGS]           tools/fp8_bench.py ARGS
#   prof[=ARGS]          rocprofv3 --kernel-trace --stats of bench.py --steps 3 --warmup 1 ARGS
#   pmc=SCRIPT:ARGS      tools/SCRIPT (a rocprofv3 --pmc recipe) ARGS
#   py=FILE[:ARGS]       python FILE ARGS
#   smoke                __graft_entry__.smoke()
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
run() {  # run LIMIT LOG cmd...
  local lim=$1 log=$2; shift 2
  echo "== $(date +%T) $*" | tee -a gpurun_out/${TAG}_steps.txt
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a gpurun_out/${TAG}_steps.txt
  grep -v amdgpu.ids "$log" | tail -n 40
  if [ $rc -ne 0 ]; then echo "stopping: step failed rc=$rc"; exit $rc; fi
}
i=0
for step in "$@"; do
  i=$((i + 1))
  name=${step%%=*}; arg=${step#*=}; [ "$arg" = "$step" ] && arg=""
  log=gpurun_out/${TAG}_${i}_${name}.log
  case $name in
    tests) ta=${arg:-tests}; run 1000 $log python -u -m pytest ${ta//,/ } -m gpu -x -q -s -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    bench) run 600 $log python bench.py ${arg//,/ } ;;
    gemm) GEMM_VARIANTS=${arg%%:*} run 600 $log python tools/gemm_bench.py $(echo ${arg#*:} | tr , ' ') ;;
    attn) run 300 $log python tools/attn_bench.py ${arg//,/ } ;;
    fp8) run 600 $log python tools/fp8_bench.py ${arg//,/ } ;;
    prof) run 600 $log rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_prof" -o b16 -- \
            python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-sample 0 --parity-steps 0 ${arg//,/ } ;;
    pmc) run 600 $log bash tools/${arg%%:*} $(echo ${arg#*:} | tr , ' ') ;;
    py) f=${arg%%:*}; a=${arg#*:}; [ "$a" = "$arg" ] && a=""; run 600 $log python $f ${a//,/ } ;;
    smoke) run 300 $log python -c "import __graft_entry__ as g; g.smoke()" ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
echo all-ok
