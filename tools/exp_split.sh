#!/bin/bash
# Timing experiments on the split-fp16 kernels (gpurun): the default library and the
# invalid-result experiment builds (exp_*.so, default ONEPROD: the hi.hi product only), every
# sample decoded exactly (DSR_LITE=0) on one stream, one bench line each.
set -u
mkdir -p gpurun_out
C=dsp-slam-rgbd_amd/csrc
for v in base ${EXPS:-ONEPROD}; do
  lib=$C/libdsr.so; [ $v = base ] || lib=$C/exp_$v.so
  DSR_LIB=$(pwd)/$lib DSR_LITE=0 DSR_STREAMS=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 \
    --no-extra --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/exps_$v.json 2> gpurun_out/exps_$v.err
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
