# round 6: chunked render passes for multi-group batches (DSR_PRESCAN=1) vs the per-object pass
# kernel, bench main leg twice each (interleaved), + a kernel trace of the single call
set -u
mkdir -p gpurun_out
T=${1:-r6z}
for i in 1 2; do
  for P in 0 1; do
    DSR_PRESCAN=$P timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-extra --no-config4 \
      > gpurun_out/${T}_bench_p${P}_$i.log 2>&1 || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${T}_single -o run -- \
  python -u tools/single_call.py --reps 8 > gpurun_out/${T}_single_prof.log 2>&1
