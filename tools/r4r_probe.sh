#!/bin/bash
# r4r: tile tables written by the whole block (tile_scan) — A = previous build (exp_head.so),
# B = this tree's libdsr.so: bitwise signature, then one KITTI object per call, the keyframe
# stream and the 8-object shard, alternating A / B twice.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
A=$R/dsp-slam-rgbd_amd/csrc/exp_head.so; B=$R/dsp-slam-rgbd_amd/csrc/libdsr.so
DSR_LIB=$A timeout -k 10 150 python tools/batch_sig.py gpurun_out/r4r_sigA.npz > gpurun_out/r4r_sig.log 2>&1 || exit 1
DSR_LIB=$B timeout -k 10 150 python tools/batch_sig.py gpurun_out/r4r_sigB.npz >> gpurun_out/r4r_sig.log 2>&1 || exit 1
python tools/batch_sig.py --compare gpurun_out/r4r_sigA.npz gpurun_out/r4r_sigB.npz | tee -a gpurun_out/r4r_sig.log
for rep in 1 2; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    DSR_LIB=$lib timeout -k 10 120 python tools/single_call.py --reps 30 > gpurun_out/r4r_single_${v}${rep}.txt 2>&1 || exit 1
    echo "single $v$rep: $(tail -1 gpurun_out/r4r_single_${v}${rep}.txt)"
    DSR_LIB=$lib timeout -k 10 150 python tools/keyframe_bench.py > gpurun_out/r4r_kf_${v}${rep}.txt 2>&1 || exit 1
    echo "keyframe $v$rep: $(tail -1 gpurun_out/r4r_kf_${v}${rep}.txt)"
    DSR_LIB=$lib timeout -k 10 150 python bench.py --objects 8 --steps 20 --warmup 2 --no-extra --no-cpu-baseline \
      --no-config4 > gpurun_out/r4r_o8_${v}${rep}.json 2> gpurun_out/r4r_o8_${v}${rep}.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/r4r_o8_${v}${rep}.json').read().strip().splitlines()[-1]);print('o8 $v$rep', round(d['value'],1), round(d['ms_per_step'],3))"
  done
done
