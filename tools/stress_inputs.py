"""Write the input files of examples/dsr_c_stress.c / dsr_c_smoke.c (weights.f32, params.f32,
objects.bin) without a GPU: the folded bench decoder, KITTI parameters at 3 iterations, 5
KITTI-like objects of 512 points — what tests/test_gpu_api.py's stress tests write.
    python tools/stress_inputs.py <dir>"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "dsp-slam-rgbd_amd"), REPO]
import synthetic as S  # noqa: E402
from deep_sdf.workspace import fold_state  # noqa: E402

d = sys.argv[1]
os.makedirs(d, exist_ok=True)
layers = fold_state(S.make_decoder(1234), S.DEFAULT_SPECS)
np.concatenate([np.concatenate([W.reshape(-1), b.reshape(-1)]) for W, b in layers]).astype(np.float32).tofile(
    os.path.join(d, "weights.f32"))
jo = S.KITTI_OPTIM["joint_optim"]
np.array([jo["k1"], jo["k2"], jo["k3"], jo["k4"], jo["b1"], jo["b2"], jo["learning_rate"], jo["scale_damping"], 3,
          S.KITTI_OPTIM["code_len"], S.KITTI_OPTIM["num_depth_samples"], S.KITTI_OPTIM["cut_off_threshold"],
          S.KITTI_OPTIM.get("pose_only_optim", {"num_iterations": 5})["num_iterations"]],
         np.float32).tofile(os.path.join(d, "params.f32"))
objs = [S.kitti_object(i, base_seed=1000, n_pts=512) for i in range(5)]
with open(os.path.join(d, "objects.bin"), "wb") as fh:
    fh.write(np.int32(len(objs)).tobytes())
    for o in objs:
        fh.write(np.array([o.pts.shape[0], o.rays.shape[0], o.depth.shape[0]], np.int32).tobytes())
        for a in (o.t_cam_obj, o.pts, o.rays, o.depth):
            fh.write(np.ascontiguousarray(a, np.float32).tobytes())
