#!/bin/bash
# One gpurun call: GPU tests, then (only if the tests ended normally, pass or fail) the
# default bench, the small-shard sweep and the round profile.  Stops at the first GPU
# step that times out, aborts or faults (exit codes other than 0/1 for pytest, 0 else).
set -u
TAG=${1:-r2}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
[ "${SWEEP:-1}" = 1 ] && { bash tools/scale_sweep.sh ${TAG}_sweep || exit $?; }
[ "${PROFILE:-1}" = 1 ] && { bash tools/profile_round.sh ${TAG} > gpurun_out/${TAG}_profile.log 2>&1; echo "profile rc=$?"; }
exit 0
