#!/bin/bash
# r4v: the ens256 per-iteration test on kitti0 / kitti5 with the shipped fp64 rotation prior and
# with the reference's fp32 chain (experiment build exp_prior32.so)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in prior32 shipped; do
  lib=$R/dsp-slam-rgbd_amd/csrc/libdsr.so; [ $v = prior32 ] && lib=$R/dsp-slam-rgbd_amd/csrc/exp_prior32.so
  DSR_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_contract.py -m gpu -v -s --timeout 240 \
    --timeout-method thread -k "ens256" > gpurun_out/r4v_$v.log 2>&1
  echo "$v rc=$?"; grep -E "^it [0-9]|ens256_distribution.*it 0|oracle's|smallest|passed|failed" gpurun_out/r4v_$v.log | cut -c1-160
done
