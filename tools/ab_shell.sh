#!/bin/bash
# Audit shell A/B: the lite-audit GPU tests, then the default bench workload with
# DSR_LITE_SHELL=0 (no certain audit beyond the band: the shipped behaviour before round 3's fix)
# and 1 (band edge + one margin, th + 2m), two alternating rounds, then tools/lite_audit_all.py
# (every lite sample re-decoded exactly).  Run through gpurun from the repo root.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lite_audit.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "audit or lite or early_ray or refine or calibrated or hooks or query or graph_replays_redo" > gpurun_out/shell_tests.log 2>&1 || exit $?
for r in 1 2; do
  for sh in 0 1; do
    DSR_LITE_SHELL=$sh timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra --no-config4 > gpurun_out/shell_ab_${sh}_$r.json 2>/dev/null || exit $?
  done
done
timeout -k 10 600 python -u tools/lite_audit_all.py 6 > gpurun_out/audit_all.txt 2>&1
