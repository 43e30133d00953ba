#!/bin/bash
# Profile the default bench workload on the GPU box (run through gpurun from the repo root).
# Writes gpurun_out/prof_<tag>/ (kernel trace + stats) and one PMC pass per counter.
set -u
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_$TAG -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra --no-config4 > $R/gpurun_out/prof_$TAG.log 2>&1 || exit 1
# the same workload on one stream: per-kernel durations without the other object group's
# concurrent kernels in them (the default run overlaps two groups)
DSR_STREAMS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_${TAG}_s1 -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra --no-config4 > $R/gpurun_out/prof_${TAG}_s1.log 2>&1 || exit 1
CTRS=${CTRS:-FETCH_SIZE WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F32 TCC_HIT_sum TCC_MISS_sum SQ_BUSY_CYCLES}
for C in $CTRS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -f csv -d $R/gpurun_out/pmc_${TAG}_$C -o pmc -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extra --no-config4 > $R/gpurun_out/pmc_${TAG}_$C.log 2>&1 || exit 1
done
cd $R && python3 tools/prof_summary.py $TAG gpurun_out/prof_$TAG gpurun_out/pmc_${TAG}_* && \
  python3 tools/prof_summary.py ${TAG}_s1 gpurun_out/prof_${TAG}_s1
