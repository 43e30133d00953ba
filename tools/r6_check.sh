# round 6: k_solve phase clock (exp_solveprof.so, -DDSR_SOLVE_PROFILE) + single-call time, then the GPU suite
set -u
mkdir -p gpurun_out
T=${1:-r6p}
L=$PWD/dsp-slam-rgbd_amd/csrc
DSR_LIB=$L/exp_solveprof.so timeout -k 10 120 python -u tools/single_call.py --reps 6 > gpurun_out/${T}_prof.log 2>&1 || exit $?
DSR_LIB=$L/libdsr.so timeout -k 10 120 python -u tools/single_call.py --reps 40 > gpurun_out/${T}_single.log 2>&1 || exit $?
DSR_LIB=$L/libdsr.so timeout -k 10 120 python -u tools/single_call.py --reps 40 >> gpurun_out/${T}_single.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
echo "tests rc=$?"
