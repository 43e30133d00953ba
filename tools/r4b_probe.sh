#!/bin/bash
# r4b: (1) leak attribution of the capacity section (host ASan build, full LeakSanitizer report);
# (2) lite-kernel HBM traffic, r2y library vs HEAD, one stream, per-dispatch FETCH/WRITE_SIZE;
# (3) the two tests that failed on r4a.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
python3 tools/stress_inputs.py gpurun_out/stress_in || exit 1
CS=$R/dsp-slam-rgbd_amd/csrc
for skip in "graph,trace,resident,redo,multi,query,mesher,errors" "graph,trace,resident,redo,multi,query,mesher,errors,capacity"; do
  ASAN_OPTIONS=detect_leaks=1 DSR_STRESS_SKIP=$skip timeout -k 10 200 $CS/dsr_c_stress_asan gpurun_out/stress_in \
    > gpurun_out/leak_$(echo $skip | tr -cd 'a-z' | tail -c 8).txt 2>&1
  echo "leak run rc=$?"
done
export TMPDIR=/tmp
for tree in head r2y; do
  if [ $tree = head ]; then B="$R/bench.py --no-config4"; else B="$R/exp_r2y/bench.py"; fi
  for C in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && DSR_STREAMS=1 timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $C -f csv -d $R/gpurun_out/tab_${tree}_$C -o pmc -- \
      python3 $B --steps 1 --warmup 0 --no-cpu-baseline --no-extra > $R/gpurun_out/tab_${tree}_$C.log 2>&1)
    rc=$?; echo "pmc $tree $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_lite_audit.py tests/test_gpu_api.py -m gpu -v --timeout 300 \
  --timeout-method thread -k "high_error or leaks or bench_decoder" > gpurun_out/r4b_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/r4b_tests.log
