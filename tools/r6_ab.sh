# round 6: GPU suite, then alternating bench lines of the shipped library and an experiment build
# (one-stream kernel durations: bench.py rooflines_one_stream).  usage: bash tools/r6_ab.sh TAG EXP.so
set -u
mkdir -p gpurun_out
T=$1; X=$2
L=$PWD/dsp-slam-rgbd_amd/csrc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for lib in libdsr.so $X; do
    DSR_LIB=$L/$lib timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/${T}_${lib%.so}_$r.json 2> gpurun_out/${T}_${lib%.so}_$r.err || exit $?
  done
done
