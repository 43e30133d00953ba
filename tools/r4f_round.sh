#!/bin/bash
# r4f: final full GPU suite, smoke(), bench at the end of round 4
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread --maxfail=10 \
  > gpurun_out/r4f_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r4f_suite.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.log 2>&1
echo "smoke rc=$?"; tail -1 gpurun_out/r4f_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r4f_bench.json 2> gpurun_out/r4f_bench.err
echo "bench rc=$?"; tail -c 300 gpurun_out/r4f_bench.err
