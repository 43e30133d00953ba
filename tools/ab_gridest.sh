#!/bin/bash
# (the DSR_GRID_EST switch existed only in that experiment build; measured and removed)
# A/B of DSR_GRID_EST (exact-pass / Jacobian grids from a host tile estimate) on one box:
# bitwise signature, then alternating 8-object shard benches and keyframe batches.
set -u
mkdir -p gpurun_out
DSR_GRID_EST=0 timeout -k 10 120 python tools/batch_sig.py gpurun_out/ge_sig0.npz > gpurun_out/ge_sig.log 2>&1 || exit 1
DSR_GRID_EST=1 timeout -k 10 120 python tools/batch_sig.py gpurun_out/ge_sig1.npz >> gpurun_out/ge_sig.log 2>&1 || exit 1
python tools/batch_sig.py --compare gpurun_out/ge_sig0.npz gpurun_out/ge_sig1.npz >> gpurun_out/ge_sig.log 2>&1
for rep in 1 2 3; do
  for v in 0 1; do
    DSR_GRID_EST=$v timeout -k 10 200 python bench.py --objects 8 --steps 10 --warmup 2 --no-extra --no-cpu-baseline \
      > gpurun_out/ge_o8_${v}_${rep}.json 2> /dev/null || exit 1
    DSR_GRID_EST=$v timeout -k 10 200 python tools/keyframe_bench.py > gpurun_out/ge_kf_${v}_${rep}.log 2>&1 || exit 1
  done
done
