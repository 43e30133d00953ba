#!/bin/bash
# One GPU call: the -m gpu suite, then (unless the suite crashed) one bench run.
# usage: tools/gpu_suite_bench.sh TAG [bench args...]
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --maxfail=10 \
  > gpurun_out/${tag}_suite.log 2>&1
rc=$?
echo "suite rc=$rc"; tail -5 gpurun_out/${tag}_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python bench.py "$@" > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
brc=$?
echo "bench rc=$brc"; tail -c 600 gpurun_out/${tag}_bench.err
exit $brc
