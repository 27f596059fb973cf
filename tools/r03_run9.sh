# two-stream CU sharing A/B: persistent 4-wave grid cap, and serial towers
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 224 192 160; do
  CLIPMI_W4P_GRID=$v timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/r03r9_g$v.json 2> gpurun_out/r03r9_g$v.err || { echo "bench $v failed"; tail -5 gpurun_out/r03r9_g$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03r9_g$v.json')); print('grid $v', d['value'], d['ms_per_step'])"
done
CLIPMI_OVERLAP=0 timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/r03r9_serial.json 2> gpurun_out/r03r9_serial.err || { echo "serial failed"; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r03r9_serial.json')); print('serial', d['value'], d['ms_per_step'])"
