#!/bin/bash
# Kernel trace of the config-5 keyframe batch (8 Redwood hypotheses, 5 iterations, re-run
# back to back; tools/keyframe_bench.py) for one library or two (gpurun).
# usage: bash tools/trace_kf.sh TAG [LIB ...]   -> gpurun_out/trace_kf_<TAG><i>/
set -u
TAG=$1; shift
R=$(pwd)
export TMPDIR=/tmp
i=0
for lib in "${@:-dsp-slam-rgbd_amd/csrc/libdsr.so}"; do
  (cd /tmp && DSR_LIB=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/trace_kf_${TAG}$i -o run -- \
    python3 $R/tools/keyframe_bench.py --reps 10 > $R/gpurun_out/trace_kf_${TAG}$i.log 2>&1) || exit 1
  i=$((i + 1))
done
