#!/bin/bash
# r4i: LayerNorm decoders + variant instantiations: the shipped decoder bitwise unchanged
# (signature vs the previous build), the variant tests, the full GPU suite (ensemble
# per-iteration test deselected until its criterion lands), smoke(), the driver's bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
# (the signature is compared here against r4g's, the previous ABI's build, on the CPU side)
timeout -k 10 400 python3 -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_variants.py \
  > gpurun_out/r4i_var.log 2>&1
echo "variants rc=$?"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r4i_var.log | tail -16
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --maxfail=10 \
  --deselect tests/test_gpu_contract.py::test_ens256_distribution_per_iteration > gpurun_out/r4i_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r4i_suite.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4i_smoke.log 2>&1
echo "smoke rc=$?"; tail -2 gpurun_out/r4i_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r4i_bench.json 2> gpurun_out/r4i_bench.err
echo "bench rc=$?"; tail -c 300 gpurun_out/r4i_bench.err
