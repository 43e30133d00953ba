#!/bin/bash
# r4d: code-32 GPU tests after the lin4/lin3^T depth fix, the accuracy probe (split vs fp32
# MFMA vs fp64 truth; per-iteration ensemble table), then the fp64 / ensemble tests.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_code32.py \
  > gpurun_out/r4d_code32.log 2>&1
echo "code32 rc=$?"; grep -E "passed|failed|Error|assert" gpurun_out/r4d_code32.log | tail -8
timeout -k 10 400 python3 -u tools/acc_probe.py > gpurun_out/r4d_acc.json 2> gpurun_out/r4d_acc.log
rc=$?; echo "acc rc=$rc"; cat gpurun_out/r4d_acc.log | tail -30
