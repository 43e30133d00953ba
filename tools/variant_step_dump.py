"""Teacher-forced GN steps of a decoder variant (golden F17 states) on the GPU — H, b, dx, K per
recorded state — for offline comparison with the fp64 oracle (diagnostic; GPU box).
usage: [DSR_LIB=...] python tools/variant_step_dump.py ln TAG -> gpurun_out/variant_step_<v>_<TAG>.npz"""
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import synthetic as S  # noqa: E402
from conftest import golden, make_cfg  # noqa: E402
from deep_sdf.workspace import decoder_from_state  # noqa: E402
from reconstruct.optimizer import Optimizer  # noqa: E402
from test_oracle_golden import _variant_specs  # noqa: E402

v, tag = sys.argv[1], sys.argv[2]
f = golden("f17_variants.npz")
dec = decoder_from_state(S.make_decoder(1234, _variant_specs(v)), _variant_specs(v))
K3 = dict(S.KITTI_OPTIM, joint_optim=dict(S.KITTI_OPTIM["joint_optim"], num_iterations=1))
opt = Optimizer(dec, make_cfg(K3, "KITTI"))
n_it = int(f[v + "_n_iters_run"])
objs = [(f[v + "_it_t_obj_cam"][e], f[v + "_obj_pts"], f[v + "_obj_rays"], f[v + "_obj_depth"], f[v + "_it_z"][e])
        for e in range(n_it)]
_, tr = opt.reconstruct_objects(objs, trace=True, pose_is_obj_cam=True)
np.savez_compressed(os.path.join(REPO, "gpurun_out", f"variant_step_{v}_{tag}.npz"),
                    **{k: np.array([t[k][0] for t in tr]) for k in ("H", "b", "dx", "k", "loss")})
print("done")
