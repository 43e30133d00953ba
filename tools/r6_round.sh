set -u
mkdir -p gpurun_out
L=$PWD/dsp-slam-rgbd_amd/csrc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r6j_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
DSR_LIB=$L/exp_r5head.so timeout -k 10 200 python -u tools/batch_sig.py gpurun_out/r6j_sig_head.npz > gpurun_out/r6j_sig.log 2>&1 || exit $?
DSR_LIB=$L/libdsr.so timeout -k 10 200 python -u tools/batch_sig.py gpurun_out/r6j_sig_new.npz >> gpurun_out/r6j_sig.log 2>&1 || exit $?
python tools/batch_sig.py --compare gpurun_out/r6j_sig_head.npz gpurun_out/r6j_sig_new.npz >> gpurun_out/r6j_sig.log 2>&1
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/r6j_bench.json 2> gpurun_out/r6j_bench.err
echo "bench rc=$?"
