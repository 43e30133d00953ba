#!/bin/bash
# r5b: raw MFMA rounding data + signed decoder error (bias) of the fp32 and split kernels
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/mfma_numerics.py 1 > gpurun_out/r5b_mfma.log 2>&1; rc=$?; echo "mfma rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bias_probe.py > gpurun_out/r5b_bias.log 2>&1; rc=$?; echo "bias rc=$rc"; exit $rc
