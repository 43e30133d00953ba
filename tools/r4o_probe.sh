#!/bin/bash
# r4o: the HIP runtime alone under host ASan — does its exit-time teardown trip the sanitizer?
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
ASAN_OPTIONS=detect_leaks=0 timeout -k 10 120 dsp-slam-rgbd_amd/csrc/hip_asan_teardown > gpurun_out/r4o_probe.log 2>&1
echo "rc=$?"; head -c 3000 gpurun_out/r4o_probe.log
