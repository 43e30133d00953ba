#!/bin/bash
# Kernel traces for timeline analysis (gpurun): the 8-object strong-scaling shard and the
# 64-object bench on one stream (per-launch durations of every render pass).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/trace_o8 -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --objects 8 > $R/gpurun_out/trace_o8.log 2>&1 || exit 1
DSR_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/trace_o64s1 -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra > $R/gpurun_out/trace_o64s1.log 2>&1
