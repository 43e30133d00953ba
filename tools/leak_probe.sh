#!/bin/bash
# LeakSanitizer attribution for examples/dsr_c_stress.c (host-ASan build): direct-leak
# summaries with each stress section left out, against context + decoder only (GPU box).
mkdir -p gpurun_out
timeout -k 10 120 python -c "
import sys; sys.path[:0]=['dsp-slam-rgbd_amd','tests']
import pathlib, numpy as np, synthetic as S
from deep_sdf.workspace import decoder_from_state
from reconstruct.optimizer import Optimizer
from conftest import make_cfg
d=pathlib.Path('gpurun_out/stress_in'); d.mkdir(exist_ok=True)
dec=decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS, device=0)
opt=Optimizer(dec, make_cfg(dict(S.KITTI_OPTIM, joint_optim=dict(S.KITTI_OPTIM['joint_optim'], num_iterations=3)), 'KITTI'))
import test_gpu_api as T
T._write_c_inputs(d, dec, opt, [S.kitti_object(i, base_seed=1000, n_pts=512) for i in range(5)])
print('inputs ok')
" > gpurun_out/leak_probe.log 2>&1 || exit 1
run() {   # label, env...
  echo "== $1" >> gpurun_out/leak_probe.log; shift
  env "$@" ASAN_OPTIONS=detect_leaks=1 timeout -k 10 120 dsp-slam-rgbd_amd/csrc/dsr_c_stress_asan gpurun_out/stress_in >> gpurun_out/leak_probe.log 2>&1
  echo "rc=$?" >> gpurun_out/leak_probe.log
}
run minimal DSR_STRESS_MINIMAL=1
run full DSR_STRESS_MINIMAL=0
for sec in trace resident redo graph multi query mesher errors; do run "skip-$sec" DSR_STRESS_SKIP=$sec; done
run skip-all DSR_STRESS_SKIP=trace,resident,redo,graph,multi,query,mesher,errors
grep -E "^== |rc=|stress ok|SUMMARY|Direct leak" gpurun_out/leak_probe.log
