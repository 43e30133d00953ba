#!/bin/bash
# Per-group hipGraph replay (DSR_GRAPH=1) vs eager launches, same box: graph tests, then the
# 8- and 64-object shards and the 8 x 4096-point shard, alternating, two rounds.
set -u
TAG=${1:-abg}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lite_audit.py tests/test_gpu_parity.py -k "graph" -v \
  --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "graph tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -le 1 ] || exit $rc
run() {   # name, env..., -- bench args
  local name=$1; shift
  env "$@" > gpurun_out/${TAG}_${name}.json 2> gpurun_out/${TAG}_${name}.err
  local rc=$?
  echo "$name rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_${name}.json').read().strip().splitlines()[-1]); print(round(d['value'],1), round(d['ms_per_step'],3))" 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
}
B="python bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-config4"
for r in 1 2; do
  run o8_e$r DSR_GRAPH=0 timeout -k 10 200 $B --objects 8
  run o8_g$r DSR_GRAPH=1 timeout -k 10 200 $B --objects 8
  run p4096o8_e$r DSR_GRAPH=0 timeout -k 10 200 $B --objects 8 --pts 4096
  run p4096o8_g$r DSR_GRAPH=1 timeout -k 10 200 $B --objects 8 --pts 4096
  run o64_e$r DSR_GRAPH=0 timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-extra --no-cpu-baseline --no-config4
  run o64_g$r DSR_GRAPH=1 timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-extra --no-cpu-baseline --no-config4
done
for r in 1 2; do     # (keyframe_bench runs eager and graph itself)
  timeout -k 10 200 python tools/keyframe_bench.py > gpurun_out/${TAG}_kf$r.log 2>&1 || exit $?
  grep -E "graph=|one call" gpurun_out/${TAG}_kf$r.log
done
