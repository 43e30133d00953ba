#!/bin/bash
# r4s: the first render pass's per-ray scan over the ray chunks (k_sample_scan) and k_solve's
# panel-blocked LU — A = previous build (exp_head.so),
# B = this tree's libdsr.so: bitwise signature, then one KITTI object per call, the keyframe
# stream and the 8-object shard, alternating A / B twice.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
A=$R/dsp-slam-rgbd_amd/csrc/exp_head.so; B=$R/dsp-slam-rgbd_amd/csrc/libdsr.so
DSR_LIB=$A timeout -k 10 150 python tools/batch_sig.py gpurun_out/r4s_sigA.npz > gpurun_out/r4s_sig.log 2>&1 || exit 1
DSR_LIB=$B timeout -k 10 150 python tools/batch_sig.py gpurun_out/r4s_sigB.npz >> gpurun_out/r4s_sig.log 2>&1 || exit 1
python tools/batch_sig.py --compare gpurun_out/r4s_sigA.npz gpurun_out/r4s_sigB.npz | tee -a gpurun_out/r4s_sig.log
for rep in 1 2; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    DSR_LIB=$lib timeout -k 10 120 python tools/single_call.py --reps 30 > gpurun_out/r4s_single_${v}${rep}.txt 2>&1 || exit 1
    echo "single $v$rep: $(tail -1 gpurun_out/r4s_single_${v}${rep}.txt)"
    DSR_LIB=$lib timeout -k 10 150 python tools/keyframe_bench.py > gpurun_out/r4s_kf_${v}${rep}.txt 2>&1 || exit 1
    echo "keyframe $v$rep: $(tail -1 gpurun_out/r4s_kf_${v}${rep}.txt)"
    DSR_LIB=$lib timeout -k 10 150 python bench.py --objects 8 --steps 20 --warmup 2 --no-extra --no-cpu-baseline \
      --no-config4 > gpurun_out/r4s_o8_${v}${rep}.json 2> gpurun_out/r4s_o8_${v}${rep}.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/r4s_o8_${v}${rep}.json').read().strip().splitlines()[-1]);print('o8 $v$rep', round(d['value'],1), round(d['ms_per_step'],3))"
  done
done
for v in A B; do
  lib=$A; [ $v = B ] && lib=$B
  DSR_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-config4 \
    > gpurun_out/r4s_o64_${v}.json 2> gpurun_out/r4s_o64_${v}.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r4s_o64_${v}.json').read().strip().splitlines()[-1]);print('o64 $v', round(d['value'],1), round(d['ms_per_step'],3))"
done
DSR_SAMPLE_PRESCAN=0 timeout -k 10 120 python tools/single_call.py --reps 30 > gpurun_out/r4s_single_B_noprescan.txt 2>&1 || exit 1
echo "single B, DSR_SAMPLE_PRESCAN=0: $(tail -1 gpurun_out/r4s_single_B_noprescan.txt)"
bash tools/trace_single.sh r4s || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_api.py tests/test_gpu_contract.py > gpurun_out/r4s_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4s_tests.log; exit $rc
