"""The GPU's per-iteration (K, loss) and final state from the 256 starts of golden F13 <name>, in
one batch (GPU box) -> gpurun_out/gpu_ens_<name>.npz, for offline comparison with the
reference's (F13), the fp32 oracle's (F16) and the fp64 oracle's (F19) clouds.
Usage: python tools/gpu_ens_dump.py kitti0 kitti5   (DSR_ENS_TAG=x: gpu_ens_x_<name>.npz)"""
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import synthetic as S  # noqa: E402
from conftest import golden, make_cfg  # noqa: E402
from deep_sdf.workspace import decoder_from_state  # noqa: E402
from reconstruct.optimizer import Optimizer  # noqa: E402

TAG = os.environ.get("DSR_ENS_TAG", "")
TAG = TAG + "_" if TAG else ""
dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
opt = Optimizer(dec, make_cfg(S.KITTI_OPTIM, "KITTI"))
for name in sys.argv[1:]:
    f = golden(f"f4_traj_{name}.npz")
    e = golden(f"f13_ens256_{name}.npz")
    res, tr = opt.reconstruct_objects([(t, f["obj_pts"], f["obj_rays"], f["obj_depth"], None) for t in e["t_init"]],
                                      trace=True)
    np.savez_compressed(os.path.join(REPO, "gpurun_out", f"gpu_ens_{TAG}{name}.npz"),
                        it_k=np.array([t["k"] for t in tr]), it_loss=np.array([t["loss"] for t in tr]),
                        loss=np.array([r["loss"] for r in res]), is_good=np.array([r["is_good"] for r in res]),
                        t_cam_obj=np.array([r["t_cam_obj"] for r in res]), code=np.array([r["code"] for r in res]))
    print(name, "done")
