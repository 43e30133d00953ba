"""Teacher-forced GN steps from every recorded state of a margin-screened fixture (golden F8) and
the free-running trajectory, on the GPU — H, b, dx, K, n_valid and the trajectory's pre-update
states — for offline comparison with the fp64 oracle (diagnostic; GPU box).
usage: [DSR_LIB=...] python tools/f8_step_dump.py redwood_s5359 TAG -> gpurun_out/f8_step_<name>_<TAG>.npz"""
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import synthetic as S  # noqa: E402
from conftest import make_cfg  # noqa: E402
from deep_sdf.workspace import decoder_from_state  # noqa: E402
from reconstruct.optimizer import Optimizer  # noqa: E402
from test_gpu_contract import optim_of  # noqa: E402

name, tag = sys.argv[1], sys.argv[2]
f = np.load(os.path.join(REPO, "tests", "golden", f"f8_margin_{name}.npz"), allow_pickle=False)
optim, dtp = optim_of(f)
dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
one = dict(optim, joint_optim=dict(optim["joint_optim"], num_iterations=1))
n_it = int(f["n_iters_run"])
_, tf = Optimizer(dec, make_cfg(one, dtp)).reconstruct_objects(
    [(f["it_t_obj_cam"][e], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][e]) for e in range(n_it)],
    trace=True, pose_is_obj_cam=True)
(r,), (t,) = Optimizer(dec, make_cfg(optim, dtp)).reconstruct_objects(
    [(f["obj_t_cam_obj"], f["obj_pts"], f["obj_rays"], f["obj_depth"], None)], trace=True)
out = {k: np.array([x[k][0] for x in tf]) for k in ("H", "b", "dx", "k", "n_valid", "loss")}
out.update({"run_" + k: np.asarray(t[k]) for k in ("t_obj_cam", "z", "k", "n_valid", "loss", "H", "b", "dx")})
np.savez_compressed(os.path.join(REPO, "gpurun_out", f"f8_step_{name}_{tag}.npz"), **out)
print("done")
