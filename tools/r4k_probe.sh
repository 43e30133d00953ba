#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 300 python3 -u tools/ln_precision.py > gpurun_out/r4k_prec.log 2>&1
echo "rc=$?"; cat gpurun_out/r4k_prec.log | grep -v amdgpu.ids
