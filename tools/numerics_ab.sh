#!/bin/bash
# Numerics A/B of library builds on one GPU box (through gpurun, from the repo root).  For every
# variant NAME=LIB[:K=V,K=V...] (LIB relative to the repo root; the K=V pairs are exported for that
# variant's runs, e.g. DSR_TEST_HOOKS=1,DSR_SURFACE_EXACT=1): the decoder's sdf / Jacobian bias
# against fp64 (tools/bias_probe.py), the 256-member kitti5 / kitti0 ensembles
# (tools/gpu_ens_dump.py -> gpurun_out/gpu_ens_<NAME>_*.npz; rank them offline with
# tools/ens_judge.py NAME_,...), then bench lines alternated over two rounds (same box).
#   usage: bash tools/numerics_ab.sh TAG ls1=dsp-slam-rgbd_amd/csrc/libdsr.so head=exp_HEAD.so ...
# (round 5 ran its numerics experiments, r5r-r5ac in DESIGN.md §3.2, as calls of this shape)
set -u
TAG=$1; shift
mkdir -p gpurun_out
run() {   # run VARIANT-SPEC CMD...: the command with the variant's library and environment
  local spec=$1; shift
  local lib=${spec#*=}; local envs=""
  case "$lib" in *:*) envs=${lib#*:}; lib=${lib%%:*};; esac
  ( export DSR_LIB=$(pwd)/$lib
    IFS=, ; for kv in $envs; do export "$kv"; done
    "$@" )
}
for spec in "$@"; do
  name=${spec%%=*}
  run "$spec" timeout -k 10 300 python -u tools/bias_probe.py > gpurun_out/${TAG}_bias_$name.log 2>&1
  rc=$?; echo "$name bias rc=$rc"; [ $rc -eq 0 ] || exit $rc
  DSR_ENS_TAG=$name run "$spec" timeout -k 10 400 python -u tools/gpu_ens_dump.py kitti5 kitti0 > gpurun_out/${TAG}_ens_$name.log 2>&1
  rc=$?; echo "$name ens rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for spec in "$@"; do
    name=${spec%%=*}
    run "$spec" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-config4 \
      > gpurun_out/${TAG}_bench_${name}_$i.json 2> gpurun_out/${TAG}_bench_${name}_$i.err
    rc=$?; echo "$name bench $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
