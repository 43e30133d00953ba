#!/bin/bash
# One rocprofv3 PMC pass over one bench step (run through gpurun from the repo root):
#   bash tools/pmc_pass.sh <tag> "<counters>" [bench args...]
set -u
TAG=$1; CTRS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -f csv -d $R/gpurun_out/pmc_$TAG -o pmc -- \
  python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extra --no-config4 "$@" > $R/gpurun_out/pmc_$TAG.log 2>&1
