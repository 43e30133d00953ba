#!/bin/bash
set -u
mkdir -p gpurun_out
L=$PWD/dsp-slam-rgbd_amd/csrc
for v in libdsr exp_ROWONLY exp_NOSIGN; do
  DSR_LIB=$L/$v.so timeout -k 10 300 python -u tools/bias_probe.py > gpurun_out/r5i_bias_$v.log 2>&1; rc=$?; echo "bias $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
