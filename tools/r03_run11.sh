# stream sharing A/B: text tower on non-persistent GEMM kernels (CLIPMI_TEXT_NONPERSIST=1) vs default
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for v in 0 1; do
  CLIPMI_TEXT_NONPERSIST=$v timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/r03r11_np$v.json 2> gpurun_out/r03r11_np$v.err || { echo "bench $v failed"; tail -5 gpurun_out/r03r11_np$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03r11_np$v.json')); print('text_nonpersist $v rep $rep', d['value'], d['ms_per_step'])"
done
done
