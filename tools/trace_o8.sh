#!/bin/bash
# Kernel trace of a small strong-scaling shard (8 objects) for timeline analysis (gpurun).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/trace_o8 -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --objects ${OBJ:-8} > $R/gpurun_out/trace_o8.log 2>&1
