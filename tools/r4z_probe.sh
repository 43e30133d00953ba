#!/bin/bash
# r4z: which write of the chunked first-pass scan makes the decode counts timing-dependent with two
# object groups (experiment build exp_prescan.so, DSR_SAMPLE_PRESCAN: 1 = rinfo from the scan, dead
# cleared by the first pass as shipped; 3 = both from the scan; 0 = shipped; later build: 5 = rinfo
# written and read with agent-scope atomics)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=$R/dsp-slam-rgbd_amd/csrc/exp_prescan.so
for v in 1 5 1 5; do
  echo "== DSR_SAMPLE_PRESCAN=$v"
  DSR_SAMPLE_PRESCAN=$v REPS=5 MODES=0 DSR_LIB=$L timeout -k 10 150 python tools/refine_sig.py 2>&1 | grep rep | cut -c1-80 || exit 1
done
