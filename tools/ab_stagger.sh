#!/bin/bash
# Staggered exact pass (DSR_SPLIT_STAGGER=1) vs the barrier kernel on one box (gpurun):
# bitwise batch signatures, then alternating bench lines (64 and 8 objects).
set -u
mkdir -p gpurun_out
DSR_SPLIT_STAGGER=0 timeout -k 10 120 python tools/batch_sig.py gpurun_out/stg_sig0.npz > gpurun_out/stg_sig.log 2>&1 || exit 1
DSR_SPLIT_STAGGER=1 timeout -k 10 120 python tools/batch_sig.py gpurun_out/stg_sig1.npz >> gpurun_out/stg_sig.log 2>&1 || exit 1
python tools/batch_sig.py --compare gpurun_out/stg_sig0.npz gpurun_out/stg_sig1.npz | tee -a gpurun_out/stg_sig.log
STEPS=${STEPS:-5} bash tools/ab_env.sh stg "s0:DSR_SPLIT_STAGGER=0" "s1:DSR_SPLIT_STAGGER=1" "s0b:DSR_SPLIT_STAGGER=0" "s1b:DSR_SPLIT_STAGGER=1" || exit 1
BENCH_ARGS="--objects 8" STEPS=${STEPS:-5} bash tools/ab_env.sh stg8 "s0:DSR_SPLIT_STAGGER=0" "s1:DSR_SPLIT_STAGGER=1"
