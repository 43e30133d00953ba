#!/bin/bash
# r5m: 256-member ensembles, error-feedback build: without kept masks (the Jacobian kernel
# re-forwards render points), and with the fp32-MFMA Jacobian kernel
set -u
mkdir -p gpurun_out
DSR_TEST_HOOKS=1 DSR_KEEP_MASKS=0 DSR_ENS_TAG=fbnomask timeout -k 10 400 python -u tools/gpu_ens_dump.py kitti5 kitti0 > gpurun_out/r5m_ens1.log 2>&1; rc=$?; echo "ens1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
DSR_TEST_HOOKS=1 DSR_JAC_VARIANT=0 DSR_ENS_TAG=fbjac0 timeout -k 10 400 python -u tools/gpu_ens_dump.py kitti5 kitti0 > gpurun_out/r5m_ens2.log 2>&1; rc=$?; echo "ens2 rc=$rc"; exit $rc
