#!/bin/bash
# r5o: the surface points' forward in the Jacobian kernel (the path of batches > 16 objects) vs in
# the exact pass: teacher-forced step errors, and the 256-member ensembles with the surface
# points' forward forced into the exact pass
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/step_probe.py kitti5 kitti0 > gpurun_out/r5o_step.log 2>&1; rc=$?; echo "step rc=$rc"; [ $rc -eq 0 ] || exit $rc
DSR_TEST_HOOKS=1 DSR_SURFACE_EXACT=1 DSR_ENS_TAG=fb2surf timeout -k 10 400 python -u tools/gpu_ens_dump.py kitti5 kitti0 > gpurun_out/r5o_ens.log 2>&1; rc=$?; echo "ens rc=$rc"; exit $rc
