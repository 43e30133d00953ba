#!/bin/bash
# r4q: dynamic tile claiming in the persistent decoder launches (DSR_DYN_TILES, default on):
# bitwise signature on vs off, the lite tests (broken-block hook included), then alternating
# bench lines off / on.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
DSR_DYN_TILES=0 timeout -k 10 150 python tools/batch_sig.py gpurun_out/r4q_sig0.npz > gpurun_out/r4q_sig.log 2>&1 || exit 1
DSR_DYN_TILES=1 timeout -k 10 150 python tools/batch_sig.py gpurun_out/r4q_sig1.npz >> gpurun_out/r4q_sig.log 2>&1 || exit 1
python tools/batch_sig.py --compare gpurun_out/r4q_sig0.npz gpurun_out/r4q_sig1.npz | tee -a gpurun_out/r4q_sig.log
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_lite_audit.py \
  tests/test_gpu_parity.py > gpurun_out/r4q_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4q_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 0 1; do
    DSR_DYN_TILES=$v timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline \
      > gpurun_out/r4q_d${v}_${rep}.json 2> gpurun_out/r4q_d${v}_${rep}.err
    rc=$?; echo "d$v rep$rep rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python3 -c "import json;d=json.loads(open('gpurun_out/r4q_d${v}_${rep}.json').read().strip().splitlines()[-1]);print('d$v', round(d['value'],1), d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
  done
done
