#!/bin/bash
# r4e: fp64 rotation prior in k_solve — accuracy probe (split, fp32 kernels) and the parity tests
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/acc_probe.py split,fp32 > gpurun_out/r4e_acc.json 2> gpurun_out/r4e_acc.log
rc=$?; echo "acc rc=$rc"; grep -v "^{" gpurun_out/r4e_acc.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_contract.py tests/test_gpu_code32.py > gpurun_out/r4e_suite.log 2>&1
echo "suite rc=$?"; grep -E "FAILED|passed|failed" gpurun_out/r4e_suite.log | tail -12
