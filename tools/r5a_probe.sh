#!/bin/bash
# r5a: MFMA rounding probe, decoder precision, and the GPU's 256-member ensembles on the fp32-MFMA
# variants (attribution of the kitti5 accuracy gap)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/mfma_numerics.py > gpurun_out/r5a_mfma.log 2>&1; rc=$?; echo "mfma rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/diag_precision.py > gpurun_out/r5a_prec.log 2>&1; rc=$?; echo "prec rc=$rc"; [ $rc -eq 0 ] || exit $rc
for v in "fwd0 0 12" "jac0 12 0" "fp32 0 0"; do
  set -- $v
  DSR_ENS_TAG=$1 DSR_FWD_VARIANT=$2 DSR_JAC_VARIANT=$3 timeout -k 10 400 python -u tools/gpu_ens_dump.py kitti5 kitti0 \
    > gpurun_out/r5a_ens_$1.log 2>&1; rc=$?; echo "ens $1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
