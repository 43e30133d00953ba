#!/bin/bash
# A/B of stream priorities (DSR_STREAM_PRIO 0/1/2) on one box, alternating rounds: 64 objects,
# the 8-object strong-scaling shard, and the keyframe batch (tools/keyframe_bench.py).
set -u
TAG=${1:-prio}
mkdir -p gpurun_out
for rep in 1 2; do
  for p in 0 1 2; do
    DSR_STREAM_PRIO=$p timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-extra --no-cpu-baseline --no-config4 \
      > gpurun_out/${TAG}_o64_p${p}_${rep}.json 2>/dev/null || exit 1
    DSR_STREAM_PRIO=$p timeout -k 10 200 python bench.py --objects 8 --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-config4 \
      > gpurun_out/${TAG}_o8_p${p}_${rep}.json 2>/dev/null || exit 1
    DSR_STREAM_PRIO=$p timeout -k 10 200 python tools/keyframe_bench.py > gpurun_out/${TAG}_kf_p${p}_${rep}.log 2>&1 || exit 1
    echo "rep $rep prio $p done"
  done
done
TAG=$TAG python3 - <<'PY'
import glob, json, os
TAG = os.environ['TAG']
for w in ("o64", "o8"):
    for p in (0, 1, 2):
        v = [json.load(open(f))["value"] for f in sorted(glob.glob(f"gpurun_out/{TAG}_{w}_p{p}_*.json"))]
        print(w, "prio", p, " ".join(f"{x:.1f}" for x in v))
PY
