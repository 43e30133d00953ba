# A/B of the DSR_CU_SPLIT experiment (object groups on even/odd CU halves via CU-masked streams),
# measured and removed; the switch exists only in that experiment build, not in the product.
set -u
DSR_CU_SPLIT=0 timeout -k 10 120 python tools/batch_sig.py gpurun_out/cs_sig0.npz > gpurun_out/cs_sig.log 2>&1 || exit 1
DSR_CU_SPLIT=1 timeout -k 10 120 python tools/batch_sig.py gpurun_out/cs_sig1.npz >> gpurun_out/cs_sig.log 2>&1 || exit 1
python tools/batch_sig.py --compare gpurun_out/cs_sig0.npz gpurun_out/cs_sig1.npz >> gpurun_out/cs_sig.log 2>&1
for rep in 1 2; do for v in 0 1; do
  DSR_CU_SPLIT=$v timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/cs_o64_${v}_$rep.json 2>/dev/null || exit 1
  DSR_CU_SPLIT=$v DSR_STREAMS=2 timeout -k 10 200 python bench.py --objects 8 --steps 10 --warmup 2 --no-extra --no-cpu-baseline > gpurun_out/cs_o8_${v}_$rep.json 2>/dev/null || exit 1
done; done
