#!/bin/bash
# r5e: sign-alternated split rows (libdsr.so) vs unsigned (exp_NOSIGN.so): decoder bias, the
# 256-member ensembles, bench A/B
set -u
mkdir -p gpurun_out
L=$PWD/dsp-slam-rgbd_amd/csrc
timeout -k 10 300 python -u tools/bias_probe.py > gpurun_out/r5e_bias_sign.log 2>&1; rc=$?; echo "bias sign rc=$rc"; [ $rc -eq 0 ] || exit $rc
DSR_LIB=$L/exp_NOSIGN.so timeout -k 10 300 python -u tools/bias_probe.py > gpurun_out/r5e_bias_nosign.log 2>&1; rc=$?; echo "bias nosign rc=$rc"; [ $rc -eq 0 ] || exit $rc
DSR_ENS_TAG=sg timeout -k 10 400 python -u tools/gpu_ens_dump.py kitti5 kitti0 > gpurun_out/r5e_ens_sg.log 2>&1; rc=$?; echo "ens rc=$rc"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-config4 > gpurun_out/r5e_bench_sign_$i.json 2> gpurun_out/r5e_bench_sign_$i.err; rc=$?; echo "bench sign rc=$rc"; [ $rc -eq 0 ] || exit $rc
  DSR_LIB=$L/exp_NOSIGN.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-config4 > gpurun_out/r5e_bench_nosign_$i.json 2> gpurun_out/r5e_bench_nosign_$i.err; rc=$?; echo "bench nosign rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
