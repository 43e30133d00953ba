# round 6: 8-object shard (the N=8 strong-scaling per-GPU load), chunked passes on / off
set -u
mkdir -p gpurun_out
T=${1:-r6aa}
for i in 1 2; do
  for P in 0 1; do
    DSR_PRESCAN=$P timeout -k 10 300 python -u bench.py --objects 8 --steps 20 --warmup 3 --no-cpu-baseline --no-extra --no-config4 \
      > gpurun_out/${T}_b8_p${P}_$i.log 2>&1 || exit $?
  done
done
