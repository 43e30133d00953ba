#!/bin/bash
# r4w: the ensemble tests (kitti0 oracle yardstick; kitti0 / kitti5 against exact arithmetic)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_contract.py -m gpu -v -s --timeout 240 --timeout-method thread \
  -k "ens256 or exact_arithmetic" > gpurun_out/r4w_ens.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "worst|FAILED|PASSED|passed|failed|Error" gpurun_out/r4w_ens.log | cut -c1-200 | tail -12; exit $rc
