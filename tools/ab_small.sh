#!/bin/bash
# A/B of two library builds on one box for small and large batches (gpurun): bitwise
# signature of each, then alternating bench lines at 8 objects (strong-scaled shard size)
# and at the default 64 objects with the keyframe leg.
# usage: bash tools/ab_small.sh TAG A.so B.so   (paths relative to the repo root)
set -u
TAG=$1; A=$(pwd)/$2; B=$(pwd)/$3
mkdir -p gpurun_out
DSR_LIB=$A timeout -k 10 120 python tools/batch_sig.py gpurun_out/${TAG}_sigA.npz > gpurun_out/${TAG}_sig.log 2>&1 || exit 1
DSR_LIB=$B timeout -k 10 120 python tools/batch_sig.py gpurun_out/${TAG}_sigB.npz >> gpurun_out/${TAG}_sig.log 2>&1 || exit 1
python tools/batch_sig.py --compare gpurun_out/${TAG}_sigA.npz gpurun_out/${TAG}_sigB.npz | tee -a gpurun_out/${TAG}_sig.log
for rep in 1 2; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    DSR_LIB=$lib timeout -k 10 200 python bench.py --objects 8 --steps 10 --warmup 2 --no-extra --no-cpu-baseline \
      > gpurun_out/${TAG}_o8_${v}${rep}.json 2> gpurun_out/${TAG}_o8_${v}${rep}.err
    rc=$?; echo "o8 $v$rep rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
for rep in 1 2; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    DSR_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline \
      > gpurun_out/${TAG}_${v}${rep}.json 2> gpurun_out/${TAG}_${v}${rep}.err
    rc=$?; echo "o64 $v$rep rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
