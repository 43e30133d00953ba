#!/bin/bash
# First render window sized to one round of lite tiles: one KITTI object per
# reconstruct_object call with the fixed 16,24 schedule vs the default, two alternating rounds.
set -u
mkdir -p gpurun_out
for r in 1 2; do
  DSR_RENDER_PASSES=16,24 timeout -k 10 120 python tools/single_call.py --reps 30 > gpurun_out/abw_fixed_$r.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/single_call.py --reps 30 > gpurun_out/abw_default_$r.txt 2>&1 || exit 1
done
