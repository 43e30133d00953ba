#!/bin/bash
# Kernel traces + stats of the small batches (gpurun): the 8-object strong-scaling shard at
# 2048 and 4096 points (BASELINE configs[3] per GPU at N = 8) and the config-5 keyframe batch.
# -> gpurun_out/prof_<TAG>_{o8,p4096o8,kf}/ ; summarise here with tools/prof_summary.py and
#    tools/timeline_summary.py.
set -u
TAG=${1:-r2v}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_${TAG}_o8 -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --objects 8 \
  > $R/gpurun_out/prof_${TAG}_o8.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_${TAG}_p4096o8 -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --objects 8 --pts 4096 \
  > $R/gpurun_out/prof_${TAG}_p4096o8.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_${TAG}_kf -o run -- \
  python3 $R/tools/keyframe_bench.py --reps 10 > $R/gpurun_out/prof_${TAG}_kf.log 2>&1 || exit $?
exit 0
