#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 900 python3 -u tools/asan_teardown_probe.py > gpurun_out/r4p_asan.log 2>&1
echo "rc=$?"; grep "^==" gpurun_out/r4p_asan.log
