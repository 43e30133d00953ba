#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/mfma_bias.py > gpurun_out/r5c_mfma_bias.log 2>&1; rc=$?; echo "bias rc=$rc"; exit $rc
