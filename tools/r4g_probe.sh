#!/bin/bash
# r4g: decoder variants (use_tanh, xyz_in_all, plain Linear) on the GPU, the shipped decoder's
# results bitwise unchanged (signature vs the previous build), then the parity suite.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
timeout -k 10 120 python tools/batch_sig.py gpurun_out/r4g_sigB.npz > gpurun_out/r4g_sig.log 2>&1 || exit 1
DSR_LIB=$R/dsp-slam-rgbd_amd/csrc/exp_spill.so timeout -k 10 120 python tools/batch_sig.py gpurun_out/r4g_sigA.npz >> gpurun_out/r4g_sig.log 2>&1 || exit 1
python tools/batch_sig.py --compare gpurun_out/r4g_sigA.npz gpurun_out/r4g_sigB.npz
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_variants.py \
  > gpurun_out/r4g_var.log 2>&1
echo "variants rc=$?"; grep -E "PASSED|FAILED|passed|failed|Error|assert" gpurun_out/r4g_var.log | tail -15
timeout -k 10 600 python3 -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_code32.py > gpurun_out/r4g_par.log 2>&1
echo "parity rc=$?"; grep -E "FAILED|passed|failed" gpurun_out/r4g_par.log | tail -12
