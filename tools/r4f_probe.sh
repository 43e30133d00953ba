#!/bin/bash
# r4f: lite kernel without the per-tile spills (accumulators start as a bias copy) vs the
# previous build: bitwise signature + alternating bench lines, then one-stream PMC
# FETCH_SIZE / WRITE_SIZE of both (DESIGN.md §3.7 traffic).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
STEPS=5 bash tools/ab_lib.sh r4f dsp-slam-rgbd_amd/csrc/exp_spill.so dsp-slam-rgbd_amd/csrc/libdsr.so || exit $?
for lib in exp_spill libdsr; do
  for C in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && DSR_LIB=$R/dsp-slam-rgbd_amd/csrc/$lib.so DSR_STREAMS=1 timeout -s KILL 180 rocprofv3 --kernel-trace \
      --pmc $C -f csv -d $R/gpurun_out/tf_${lib}_$C -o pmc -- \
      python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extra --no-config4 > $R/gpurun_out/tf_${lib}_$C.log 2>&1)
    rc=$?; echo "pmc $lib $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
