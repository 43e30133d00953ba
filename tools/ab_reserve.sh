#!/bin/bash
# A/B of DSR_GRID_RESERVE (decoder grids of n_cu - k workgroups) on one box, two alternating
# rounds: 64 objects, the 8-object shard, the keyframe batch; then the batch signature of each
# setting against the default (bitwise equality).
set -u
TAG=${1:-res}
mkdir -p gpurun_out
for rep in 1 2; do
  for k in 0 8 16 32; do
    DSR_GRID_RESERVE=$k timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-extra --no-cpu-baseline --no-config4 \
      > gpurun_out/${TAG}_o64_k${k}_${rep}.json 2>/dev/null || exit 1
    DSR_GRID_RESERVE=$k timeout -k 10 200 python bench.py --objects 8 --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-config4 \
      > gpurun_out/${TAG}_o8_k${k}_${rep}.json 2>/dev/null || exit 1
    DSR_GRID_RESERVE=$k timeout -k 10 200 python tools/keyframe_bench.py > gpurun_out/${TAG}_kf_k${k}_${rep}.log 2>&1 || exit 1
    echo "rep $rep reserve $k done"
  done
done
TAG=$TAG python3 - <<'PY'
import glob, json, os, re
TAG = os.environ['TAG']
for w in ("o64", "o8"):
    for k in (0, 8, 16, 32):
        v = [json.load(open(f))["value"] for f in sorted(glob.glob(f"gpurun_out/{TAG}_{w}_k{k}_*.json"))]
        print(w, "reserve", k, " ".join(f"{x:.1f}" for x in v))
for k in (0, 8, 16, 32):
    v = [re.search(r"graph=0: .* median ([0-9.]+) ms", open(f).read()).group(1) for f in sorted(glob.glob(f"gpurun_out/{TAG}_kf_k{k}_*.log"))]
    print("kf reserve", k, " ".join(v))
PY
