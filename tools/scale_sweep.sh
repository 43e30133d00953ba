#!/bin/bash
# Per-GPU throughput of small shards (strong scaling: 64 objects / N GPUs per rank),
# run on the GPU box from the repo root; one bench per line into gpurun_out/<tag>_*.json.
set -u
TAG=${1:-sweep}
mkdir -p gpurun_out
run() {   # name, env..., -- bench args
  local name=$1; shift
  env "$@" > gpurun_out/${TAG}_${name}.json 2> gpurun_out/${TAG}_${name}.err
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run o64 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-extra --no-cpu-baseline --no-config4
run o8g DSR_GRAPH=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-extra --no-cpu-baseline --no-config4 --objects 8
run o16 timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-extra --no-cpu-baseline --no-config4 --objects 16
run o8 timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-extra --no-cpu-baseline --no-config4 --objects 8
run o8s1 DSR_STREAMS=1 timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-extra --no-cpu-baseline --no-config4 --objects 8
run o8s4 DSR_STREAMS=4 timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-extra --no-cpu-baseline --no-config4 --objects 8
run p4096o8 timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-extra --no-cpu-baseline --no-config4 --objects 8 --pts 4096
run p4096o64 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-extra --no-cpu-baseline --no-config4 --pts 4096
