#!/bin/bash
# Run GPU test files one after another; stop at the first crash (anything but pass/fail).
mkdir -p gpurun_out
for f in "$@"; do
  name=$(basename "$f" .py)
  timeout -k 10 900 python -m pytest "$f" -q -p no:cacheprovider -s ${PYTEST_X:--x} > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "$f rc=$rc" | tee -a gpurun_out/summary.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after crash rc=$rc"; exit $rc; fi
done
