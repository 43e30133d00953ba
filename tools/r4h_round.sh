#!/bin/bash
# r4h: full GPU suite (the ensemble per-iteration test deselected until its criterion lands),
# smoke(), then the driver's bench command.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --maxfail=10 \
  --deselect tests/test_gpu_contract.py::test_ens256_distribution_per_iteration > gpurun_out/r4h_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r4h_suite.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4h_smoke.log 2>&1
echo "smoke rc=$?"; tail -2 gpurun_out/r4h_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r4h_bench.json 2> gpurun_out/r4h_bench.err
echo "bench rc=$?"; tail -c 400 gpurun_out/r4h_bench.err
