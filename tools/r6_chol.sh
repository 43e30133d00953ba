# k_solve Cholesky schedule variants (round 6): per-phase clock of block 0 over 6 single calls each
set -u
mkdir -p gpurun_out
L=$PWD/dsp-slam-rgbd_amd/csrc
T=${1:-r6n}
for v in ${VARIANTS:-4 2}; do
  DSR_LIB=$L/exp_CHOL$v.so timeout -k 10 120 python -u tools/single_call.py --reps 6 > gpurun_out/${T}_chol$v.log 2>&1 || exit $?
done
