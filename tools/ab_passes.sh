#!/bin/bash
# Render-pass schedules for small batches (DSR_RENDER_PASSES): one object per
# reconstruct_object call, the 8-hypothesis Redwood keyframe batch and the 8-object KITTI shard,
# two alternating rounds (gpurun, repo root).  -> gpurun_out/abp_<spec>_<round>.txt
set -u
mkdir -p gpurun_out
for r in 1 2; do
  for spec in "16,24" "16" "0"; do
    t=$(echo "$spec" | tr ',' '-')
    {
      DSR_RENDER_PASSES=$spec timeout -k 10 120 python tools/single_call.py --reps 20 || exit 1
      DSR_RENDER_PASSES=$spec timeout -k 10 120 python tools/keyframe_bench.py --reps 20 || exit 1
      DSR_RENDER_PASSES=$spec timeout -k 10 120 python bench.py --objects 8 --steps 10 --warmup 2 --no-extra \
        --no-cpu-baseline --no-config4 || exit 1
    } > gpurun_out/abp_${t}_$r.txt 2>&1 || exit 1
  done
done
