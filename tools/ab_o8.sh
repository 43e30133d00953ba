#!/bin/bash
# Alternating A/B of two library builds on the 8-object shard (strong-scaling shard size) and
# the keyframe leg, 3 rounds.  usage: bash tools/ab_o8.sh TAG A.so B.so
set -u
TAG=$1; A=$(pwd)/$2; B=$(pwd)/$3
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    DSR_LIB=$lib timeout -k 10 200 python bench.py --objects 8 --steps 10 --warmup 2 --no-extra --no-cpu-baseline \
      > gpurun_out/${TAG}_o8_${v}${rep}.json 2> /dev/null || exit 1
    DSR_LIB=$lib timeout -k 10 200 python tools/keyframe_bench.py > gpurun_out/${TAG}_kf_${v}${rep}.log 2>&1 || exit 1
  done
done
