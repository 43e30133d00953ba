#!/bin/bash
# r4c: lite-kernel traffic bisect (PMC FETCH/WRITE_SIZE, one stream) over HEAD, a build without
# the expired-wait record (exp_NODIAG) and one without per-sample outputs (exp_NOOUT); then the
# GPU suite and a short bench on HEAD.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
for lib in libdsr exp_NODIAG exp_NOOUT; do
  for C in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && DSR_LIB=$R/dsp-slam-rgbd_amd/csrc/$lib.so DSR_STREAMS=1 timeout -s KILL 180 rocprofv3 --kernel-trace \
      --pmc $C -f csv -d $R/gpurun_out/tc_${lib}_$C -o pmc -- \
      python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extra --no-config4 > $R/gpurun_out/tc_${lib}_$C.log 2>&1)
    rc=$?; echo "pmc $lib $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 python3 tools/proto_vres.py 4096 20 > gpurun_out/r4c_proto.json 2>&1
echo "proto rc=$?"; cat gpurun_out/r4c_proto.json
tools/gpu_suite_bench.sh r4c --steps 5 --warmup 1
