#!/bin/bash
# r4n: the cross-thread release test, then the round-4 profile (tools/profile_round.sh r4n)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 300 python3 -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_api.py \
  -k "another_thread" > gpurun_out/r4n_thr.log 2>&1
echo "thread test rc=$?"; grep -E "PASSED|FAILED|Error" gpurun_out/r4n_thr.log | head -5
bash tools/profile_round.sh r4n
echo "profile rc=$?"
