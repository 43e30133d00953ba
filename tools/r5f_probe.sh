#!/bin/bash
# r5f: checkerboard signs (libdsr.so) vs row signs only (exp_ROWONLY.so): decoder bias; ensembles; bench
set -u
mkdir -p gpurun_out
L=$PWD/dsp-slam-rgbd_amd/csrc
timeout -k 10 300 python -u tools/bias_probe.py > gpurun_out/r5f_bias_cb.log 2>&1; rc=$?; echo "bias cb rc=$rc"; [ $rc -eq 0 ] || exit $rc
DSR_LIB=$L/exp_ROWONLY.so timeout -k 10 300 python -u tools/bias_probe.py > gpurun_out/r5f_bias_row.log 2>&1; rc=$?; echo "bias row rc=$rc"; [ $rc -eq 0 ] || exit $rc
DSR_ENS_TAG=cb timeout -k 10 400 python -u tools/gpu_ens_dump.py kitti5 kitti0 > gpurun_out/r5f_ens_cb.log 2>&1; rc=$?; echo "ens rc=$rc"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-config4 > gpurun_out/r5f_bench_cb_$i.json 2> gpurun_out/r5f_bench_cb_$i.err; rc=$?; echo "bench cb rc=$rc"; [ $rc -eq 0 ] || exit $rc
  DSR_LIB=$L/exp_NOSIGN.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-config4 > gpurun_out/r5f_bench_nosign_$i.json 2> gpurun_out/r5f_bench_nosign_$i.err; rc=$?; echo "bench nosign rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
