#!/bin/bash
# A/B of two library builds on one box (gpurun): bitwise signature of each, then alternating
# bench lines.  usage: bash tools/ab_lib.sh TAG A.so B.so   (paths relative to the repo root)
set -u
TAG=$1; A=$(pwd)/$2; B=$(pwd)/$3
mkdir -p gpurun_out
DSR_LIB=$A timeout -k 10 120 python tools/batch_sig.py gpurun_out/${TAG}_sigA.npz > gpurun_out/${TAG}_sig.log 2>&1 || exit 1
DSR_LIB=$B timeout -k 10 120 python tools/batch_sig.py gpurun_out/${TAG}_sigB.npz >> gpurun_out/${TAG}_sig.log 2>&1 || exit 1
python tools/batch_sig.py --compare gpurun_out/${TAG}_sigA.npz gpurun_out/${TAG}_sigB.npz | tee -a gpurun_out/${TAG}_sig.log
for rep in 1 2; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    DSR_LIB=$lib timeout -k 10 200 python bench.py --steps ${STEPS:-5} --warmup 1 --no-extra --no-cpu-baseline ${BENCH_ARGS:-} \
      > gpurun_out/${TAG}_${v}${rep}.json 2> gpurun_out/${TAG}_${v}${rep}.err
    rc=$?; echo "$v$rep rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
for v in A B; do
  lib=$A; [ $v = B ] && lib=$B
  DSR_LIB=$lib DSR_LITE=0 DSR_STREAMS=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-extra --no-cpu-baseline \
    > gpurun_out/${TAG}_${v}x.json 2> gpurun_out/${TAG}_${v}x.err
  rc=$?; echo "${v}x rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
