"""F4 at BASELINE config 4's object size: one KITTI object x 4096 surface points x
(4096+200) rays, 2 GN iterations of the REFERENCE (1 thread; build container only):

    python tests/golden/make_f4_4096.py     # writes tests/golden/f4_traj_kitti4096.npz

Same recording as make_golden.py's F4 trajectories (every iteration's state, H, b, dx,
N_valid, K), so tests/test_gpu_parity.py can teacher-force the device on each state.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, HERE)

import synthetic as S  # noqa: E402
import refshim  # noqa: E402
import make_golden as MG  # noqa: E402


def main():
    import torch

    ref = refshim.load()
    dec = refshim.build_decoder(S.make_decoder(MG.DECODER_SEED), S.DEFAULT_SPECS)
    cfg = dict(S.KITTI_OPTIM, joint_optim=dict(S.KITTI_OPTIM["joint_optim"], num_iterations=2))
    ob = S.kitti_object(0, n_pts=4096)
    r, its = MG.run_traj(ref, dec, cfg, "KITTI", ob, threads=1)
    out = MG.pack_traj(r, its)
    out.update(obj_t_cam_obj=ob.t_cam_obj, obj_pts=ob.pts, obj_rays=ob.rays, obj_depth=ob.depth,
               num_iterations=np.array(2), torch=np.array(torch.__version__))
    np.savez_compressed(os.path.join(HERE, "f4_traj_kitti4096.npz"), **out)
    print("K", out["it_k"].tolist(), "N_valid", out["it_n_valid"].tolist(), "loss", float(r.loss))


if __name__ == "__main__":
    main()
