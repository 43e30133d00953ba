#!/bin/bash
# r5d: MFMA bias regimes; decoder bias with the k-step-compensated split (libdsr.so) vs the
# single-chain accumulation (exp_NOKC.so); 256-member ensembles with the compensated build; bench A/B
set -u
mkdir -p gpurun_out
L=dsp-slam-rgbd_amd/csrc
timeout -k 10 300 python -u tools/mfma_bias.py > gpurun_out/r5d_mfma_bias.log 2>&1; rc=$?; echo "mfma rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bias_probe.py > gpurun_out/r5d_bias_kc.log 2>&1; rc=$?; echo "bias kc rc=$rc"; [ $rc -eq 0 ] || exit $rc
DSR_LIB=$PWD/$L/exp_NOKC.so timeout -k 10 300 python -u tools/bias_probe.py > gpurun_out/r5d_bias_nokc.log 2>&1; rc=$?; echo "bias nokc rc=$rc"; [ $rc -eq 0 ] || exit $rc
DSR_ENS_TAG=kc timeout -k 10 400 python -u tools/gpu_ens_dump.py kitti5 kitti0 > gpurun_out/r5d_ens_kc.log 2>&1; rc=$?; echo "ens rc=$rc"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/r5d_bench_kc_$i.json 2> gpurun_out/r5d_bench_kc_$i.err; rc=$?; echo "bench kc rc=$rc"; [ $rc -eq 0 ] || exit $rc
  DSR_LIB=$PWD/$L/exp_NOKC.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/r5d_bench_nokc_$i.json 2> gpurun_out/r5d_bench_nokc_$i.err; rc=$?; echo "bench nokc rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
