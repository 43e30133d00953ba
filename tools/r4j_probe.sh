#!/bin/bash
# r4j: the LayerNorm variant's teacher-forced and trajectory numbers (printed)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 300 python3 -u -m pytest -s -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_variants.py \
  -k "ln" > gpurun_out/r4j_var.log 2>&1
echo "rc=$?"; grep -E "^ln|PASSED|FAILED|assert" gpurun_out/r4j_var.log | head -30
