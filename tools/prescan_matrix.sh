#!/bin/bash
# DESIGN.md §3.9's reproduction matrix (GPU box, from the repo root): tools/refine_sig.py's
# 8-object batch, REPS runs per setting, the chunked first-pass scan (DSR_PRESCAN=1 test hook)
# against the shipped sequence, by group count, lite kernel, group padding and the dead-flag
# atomics build (make -C dsp-slam-rgbd_amd/csrc exp_DEADWT.so first).  Count distinct lines of
# each log:  awk '/^rep/ {print $5, $7, $9}' gpurun_out/TAG_NAME.log | sort | uniq -c
set -o pipefail
TAG=${1:-r5pm}
export DSR_TEST_HOOKS=1 MODES=0 REPS=${REPS:-16}
mkdir -p gpurun_out
LIB=$(pwd)/dsp-slam-rgbd_amd/csrc
run() {   # run NAME VAR=VALUE...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u tools/refine_sig.py > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run scan_g4 DSR_PRESCAN=1 DSR_STREAMS=4 &&
run scan_g4_lite472 DSR_PRESCAN=1 DSR_STREAMS=4 DSR_LITE_VARIANT=472 &&
run scan_g2 DSR_PRESCAN=1 DSR_STREAMS=2 &&
run scan_g1 DSR_PRESCAN=1 DSR_STREAMS=1 &&
run noscan_g4 DSR_PRESCAN=0 DSR_STREAMS=4 &&
run scan_g4_packed DSR_PRESCAN=1 DSR_STREAMS=4 DSR_GROUP_ALIGN=0 &&
{ [ ! -f $LIB/exp_DEADWT.so ] || run scan_g4_deadwt DSR_PRESCAN=1 DSR_STREAMS=4 DSR_LIB=$LIB/exp_DEADWT.so; }
