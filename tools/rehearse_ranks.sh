# rehearsal of the N>1 bench path on a one-GPU box: one RCCL rank with the process group forced on, two gloo ranks on one device
set -u
mkdir -p gpurun_out
DSR_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline --no-extra --no-config4 > gpurun_out/r6ag_force1.log 2>&1 || exit $?
DSR_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-extra --no-config4 > gpurun_out/r6ag_gloo2.log 2>&1 || exit $?
