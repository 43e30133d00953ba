# k_solve Cholesky A/B (round 6): per-phase solve clock, one object per call against the round-5
# library, then the GPU suite.  Stops at the first GPU step that does not end normally.
set -u
mkdir -p gpurun_out
T=${1:-r6k}
L=$PWD/dsp-slam-rgbd_amd/csrc
DSR_LIB=$L/exp_SOLVEPROF.so timeout -k 10 120 python -u tools/single_call.py --reps 6 > gpurun_out/${T}_solveprof.log 2>&1 || exit $?
for r in 1 2; do
  DSR_LIB=$L/exp_r5head.so timeout -k 10 120 python -u tools/single_call.py --reps 40 >> gpurun_out/${T}_single.log 2>&1 || exit $?
  DSR_LIB=$L/libdsr.so timeout -k 10 120 python -u tools/single_call.py --reps 40 >> gpurun_out/${T}_single.log 2>&1 || exit $?
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
echo "tests rc=$?"
