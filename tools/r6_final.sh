# round 6 final measurement: the driver's default bench command, then the round profile
# (kernel trace + stats on the default and one-stream workloads, one PMC pass per counter)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6_bench.json 2> gpurun_out/r6_bench.err || exit $?
bash tools/profile_round.sh r6 > gpurun_out/r6_profile.log 2>&1
echo "profile rc=$?"
