#!/bin/bash
# r5j: accumulation schemes (chain probe); sdf bias with error-feedback weight packs (libdsr.so) vs
# to-nearest packs (exp_NOFB.so); one-wave LU (exp_NOFB.so) vs round 4's LU (exp_OLDLU.so): bitwise
# signature + single-call latency; 256-member ensembles with libdsr.so
set -u
mkdir -p gpurun_out
L=$PWD/dsp-slam-rgbd_amd/csrc
timeout -k 10 200 python -u tools/split_chain_bias.py > gpurun_out/r5j_chain.log 2>&1; rc=$?; echo "chain rc=$rc"; [ $rc -eq 0 ] || exit $rc
for v in libdsr exp_NOFB; do
  DSR_LIB=$L/$v.so timeout -k 10 300 python -u tools/bias_probe.py > gpurun_out/r5j_bias_$v.log 2>&1; rc=$?; echo "bias $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
DSR_LIB=$L/exp_NOFB.so timeout -k 10 200 python -u tools/batch_sig.py gpurun_out/r5j_sig_new.npz > gpurun_out/r5j_sig.log 2>&1; rc=$?; echo "sig new rc=$rc"; [ $rc -eq 0 ] || exit $rc
DSR_LIB=$L/exp_OLDLU.so timeout -k 10 200 python -u tools/batch_sig.py gpurun_out/r5j_sig_old.npz >> gpurun_out/r5j_sig.log 2>&1; rc=$?; echo "sig old rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/batch_sig.py --compare gpurun_out/r5j_sig_new.npz gpurun_out/r5j_sig_old.npz >> gpurun_out/r5j_sig.log 2>&1; echo "compare rc=$?"
for i in 1 2; do
  DSR_LIB=$L/exp_NOFB.so timeout -k 10 200 python -u tools/single_call.py > gpurun_out/r5j_single_new_$i.log 2>&1; echo "single new rc=$?"
  DSR_LIB=$L/exp_OLDLU.so timeout -k 10 200 python -u tools/single_call.py > gpurun_out/r5j_single_old_$i.log 2>&1; echo "single old rc=$?"
done
DSR_ENS_TAG=fb timeout -k 10 400 python -u tools/gpu_ens_dump.py kitti5 kitti0 > gpurun_out/r5j_ens_fb.log 2>&1; rc=$?; echo "ens rc=$rc"; exit $rc
