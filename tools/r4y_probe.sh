#!/bin/bash
# r4y: rotation prior moved into a helper (k_solve) — bitwise signature against the previous build,
# then the parity tests that hold the prior (teacher-forced KITTI steps, fp64-accuracy, contract)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
DSR_LIB=$R/dsp-slam-rgbd_amd/csrc/exp_prev.so timeout -k 10 150 python tools/batch_sig.py gpurun_out/r4y_sigA.npz > gpurun_out/r4y_sig.log 2>&1 || exit 1
timeout -k 10 150 python tools/batch_sig.py gpurun_out/r4y_sigB.npz >> gpurun_out/r4y_sig.log 2>&1 || exit 1
python tools/batch_sig.py --compare gpurun_out/r4y_sigA.npz gpurun_out/r4y_sigB.npz || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_contract.py > gpurun_out/r4y_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4y_tests.log; exit $rc
