#!/bin/bash
# Kernel trace of back-to-back single-object reconstruct_object calls (tools/single_call.py)
# -> gpurun_out/trace_single_<TAG>/ + profiles/<TAG>_timeline.md (run through gpurun).
set -u
TAG=${1:-single}
R=$(pwd)
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/single_call.py > gpurun_out/single_${TAG}.txt 2>&1 || exit 1
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/trace_single_${TAG} -o run -- \
  python3 $R/tools/single_call.py --reps 6 > $R/gpurun_out/trace_single_${TAG}.log 2>&1) || exit 1
