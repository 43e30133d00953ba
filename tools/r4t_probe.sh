#!/bin/bash
# r4t: run-to-run determinism of the refine / decode counts with the first-pass prescan
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
B=$R/dsp-slam-rgbd_amd/csrc/libdsr.so
echo "== B 2 groups"; REPS=4 MODES=0 DSR_LIB=$B timeout -k 10 120 python tools/refine_sig.py 2>&1 | grep rep || exit 1
echo "== B 1 group"; DSR_STREAMS=1 REPS=4 MODES=0 DSR_LIB=$B timeout -k 10 120 python tools/refine_sig.py 2>&1 | grep rep || exit 1
echo "== B 2 groups, one hw queue"; GPU_MAX_HW_QUEUES=1 REPS=4 MODES=0 DSR_LIB=$B timeout -k 10 120 python tools/refine_sig.py 2>&1 | grep rep || exit 1
for v in A B; do
  DSR_LIB=$R/dsp-slam-rgbd_amd/csrc/exp_solveprof_$v.so timeout -k 10 120 python tools/single_call.py --reps 5 \
    > gpurun_out/r4t_solveprof_$v.txt 2>&1 || exit 1
  python3 - $v <<'PY'
import sys, numpy as np
v = sys.argv[1]
rows = [list(map(int, l.split()[1:4])) for l in open(f"gpurun_out/r4t_solveprof_{v}.txt") if l.startswith("solve_prof")]
a = np.array(rows[10:], float) / 100.0   # 100 MHz ticks -> us, skip the warm-up calls
print(f"solve phases {v} (us, median over {len(a)}): setup {np.median(a[:,0]):.1f} LU {np.median(a[:,1]):.1f} subst {np.median(a[:,2]):.1f}")
PY
done
