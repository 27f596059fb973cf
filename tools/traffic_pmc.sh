#!/bin/bash
# HBM traffic per launch of bench.py's roofline kernel family, from two rocprofv3 --pmc passes
# (FETCH_SIZE, WRITE_SIZE: separate runs, MI355X_MICROARCH.md "rocprofv3 PMC slots") over a
# short bench run.  Usage: tools/traffic_pmc.sh TAG  ->  gpurun_out/TAG_traffic_{wgrad,fwd_dgrad}.json (copy to profiles/)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out profiles
T=${1:-traffic}
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  CLIPMI_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/${T}_$C" -o pmc -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-sample 0 --parity-steps 0 > "$R/gpurun_out/${T}_$C.log" 2>&1 || { echo "pass $C failed rc=$?"; tail -5 "$R/gpurun_out/${T}_$C.log"; exit 1; }
done
python3 "$R/tools/traffic_summary.py" "$R/gpurun_out/${T}_FETCH_SIZE" "$R/gpurun_out/${T}_WRITE_SIZE" "$R/gpurun_out/${T}_traffic" && echo all-ok
