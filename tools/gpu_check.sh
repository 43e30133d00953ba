#!/bin/bash
# One gpurun call: GPU tests, the staggered-lite expired-wait diagnostics, the default bench.
# Stops at the first GPU step that times out, aborts or faults.
set -u
TAG=${1:-r3}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -le 1 ] || exit $rc
if [ "${DIAG:-1}" = 1 ]; then
  timeout -k 10 300 python -u tools/lite_diag.py 2 > gpurun_out/${TAG}_diag.log 2>&1
  rc=$?; echo "diag rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python bench.py --steps 5 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; exit $rc
