# round 6: 8-object shard (the N=8 per-GPU load) under render-pass windows (test hook)
set -u
mkdir -p gpurun_out
T=${1:-r6af}
for i in 1 2; do
  for P in default 12,24 20 16 16,28; do
    if [ $P = default ]; then
      timeout -k 10 300 python -u bench.py --objects 8 --steps 20 --warmup 3 --no-cpu-baseline --no-extra --no-config4 \
        > gpurun_out/${T}_${P}_$i.log 2>&1 || exit $?
    else
      DSR_TEST_HOOKS=1 DSR_RENDER_PASSES=$P timeout -k 10 300 python -u bench.py --objects 8 --steps 20 --warmup 3 \
        --no-cpu-baseline --no-extra --no-config4 > gpurun_out/${T}_${P}_$i.log 2>&1 || exit $?
    fi
  done
done
