#!/bin/bash
# A/B of runtime switches on one box: one bench line per variant into gpurun_out/<tag>_<name>.json
# usage: bash tools/ab_env.sh TAG "name1:VAR=v VAR2=v" "name2:..." ...   (run through gpurun)
set -u
TAG=$1; shift
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; vars=${spec#*:}
  env $vars timeout -k 10 200 python bench.py --steps ${STEPS:-5} --warmup 1 --no-extra --no-cpu-baseline ${BENCH_ARGS:-} \
    > gpurun_out/${TAG}_${name}.json 2> gpurun_out/${TAG}_${name}.err
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
