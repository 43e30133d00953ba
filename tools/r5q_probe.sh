#!/bin/bash
# r5q: exact (three-piece) backward weights for surface points: J systematic error, member steps,
# 256-member ensembles, bench cost
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bias_probe.py > gpurun_out/r5q_bias.log 2>&1; rc=$?; echo "bias rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/member_step_dump.py kitti5 24 > gpurun_out/r5q_member.log 2>&1; rc=$?; echo "member rc=$rc"; [ $rc -eq 0 ] || exit $rc
DSR_ENS_TAG=fb3 timeout -k 10 400 python -u tools/gpu_ens_dump.py kitti5 kitti0 > gpurun_out/r5q_ens.log 2>&1; rc=$?; echo "ens rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-config4 > gpurun_out/r5q_bench.json 2> gpurun_out/r5q_bench.err; echo "bench rc=$?"
