#!/bin/bash
# r5n: error-feedback rounding on the backward packs too (libdsr.so) vs forward packs only
# (exp_NOFB.so has neither): decoder bias / J systematic error / kink flips, ensembles, bench
set -u
mkdir -p gpurun_out
L=$PWD/dsp-slam-rgbd_amd/csrc
timeout -k 10 300 python -u tools/bias_probe.py > gpurun_out/r5n_bias.log 2>&1; rc=$?; echo "bias rc=$rc"; [ $rc -eq 0 ] || exit $rc
DSR_LIB=$L/exp_NOFB.so timeout -k 10 300 python -u tools/bias_probe.py > gpurun_out/r5n_bias_nofb.log 2>&1; rc=$?; echo "bias rc=$rc"; [ $rc -eq 0 ] || exit $rc
DSR_ENS_TAG=fb2 timeout -k 10 400 python -u tools/gpu_ens_dump.py kitti5 kitti0 > gpurun_out/r5n_ens.log 2>&1; rc=$?; echo "ens rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-config4 > gpurun_out/r5n_bench.json 2> gpurun_out/r5n_bench.err; echo "bench rc=$?"
