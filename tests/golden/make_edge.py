"""Edge-case fixtures (F10): empty and ragged inputs through the REFERENCE (build container only).

Usage::

    python tests/golden/make_edge.py        # writes tests/golden/f10_edge.npz

What the reference does (reference optimizer.py:90-205, loss.py, loss_utils.py) with inputs a
caller can hand it (the C++ side gathers points and rays per detection, so a detection can
come with few or none, src/LocalMapping_util.cc:333-391, src/Tracking_util.cc:163-200):

* ``zero_pts``  — no surface points: the sdf term is the mean of nothing, NaN
  (loss_utils.py:270) -> ``is_good False``, ``loss 0.`` at the first iteration (optimizer.py:137);
* ``zero_rays`` — no rays: fewer than 10 in-ball samples (loss.py:86-88) -> ``is_good False``;
* ``zero_both`` — both;
* ``one_pt``     — a single surface point (full trajectory);
* ``no_fg_rays`` — background rays only, no observed depth (full trajectory);
* ``no_bg_rays`` — foreground rays only (full trajectory);
* ``pose_empty`` — ``estimate_pose_cam_obj`` with no points: J^T J / 0 -> a NaN 4x4
  (optimizer.py:62-87);
* ``zhjd_empty`` — ``compute_sdf_loss_objectpoint_zhjd`` with no points: NaN (optimizer.py:207-213).

Redwood parameters, 2 GN iterations (a config value), 1 CPU thread.
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

    torch.set_num_threads(1)
    ref = refshim.load()
    dec = refshim.build_decoder(S.make_decoder(MG.DECODER_SEED), S.DEFAULT_SPECS)
    cfg = dict(S.REDWOOD_OPTIM, joint_optim=dict(S.REDWOOD_OPTIM["joint_optim"], num_iterations=2))
    ob = S.redwood_object(0, n_pts=300)
    n_fg = ob.depth.shape[0]
    cases = {
        "zero_pts": (ob.pts[:0], ob.rays, ob.depth),
        "zero_rays": (ob.pts, ob.rays[:0], ob.depth[:0]),
        "zero_both": (ob.pts[:0], ob.rays[:0], ob.depth[:0]),
        "one_pt": (ob.pts[:1], ob.rays, ob.depth),
        "no_fg_rays": (ob.pts, ob.rays[n_fg:], ob.depth[:0]),
        "no_bg_rays": (ob.pts, ob.rays[:n_fg], ob.depth),
    }
    out = {"obj_t_cam_obj": ob.t_cam_obj, "obj_pts": ob.pts, "obj_rays": ob.rays, "obj_depth": ob.depth,
           "num_iterations": np.array(2), "cases": np.array(list(cases))}
    for name, (p, r, d) in cases.items():
        o = S.SyntheticObject(ob.t_cam_obj, np.ascontiguousarray(p), np.ascontiguousarray(r),
                              np.ascontiguousarray(d), ob.t_true)
        res, its = MG.run_traj(ref, dec, cfg, "Redwood", o)
        packed = MG.pack_traj(res, its) if its and "depths" in its[0] else {
            "is_good": np.array(bool(res.is_good)), "loss": np.array(float(res.loss), np.float64),
            "n_iters_run": np.array(len(its))}
        out.update({f"{name}_{k}": v for k, v in packed.items()})
        out[f"{name}_n_pts"] = np.array(p.shape[0])
        out[f"{name}_n_rays"] = np.array(r.shape[0])
        out[f"{name}_n_fg"] = np.array(d.shape[0])
        print(name, bool(res.is_good), float(res.loss), len(its), flush=True)
    opt = refshim.make_optimizer(dec, S.KITTI_OPTIM, "KITTI")
    z = np.zeros(64, np.float32)
    T = ob.t_cam_obj.astype(np.float64)
    s = float(np.cbrt(np.linalg.det(T[:3, :3])))
    t_se3 = T.copy()
    t_se3[:3, :3] /= s
    out["pose_t_se3"] = t_se3.astype(np.float32)
    out["pose_scale"] = np.array(s, np.float32)
    out["pose_empty_out"] = np.asarray(opt.estimate_pose_cam_obj(t_se3.astype(np.float32), s, ob.pts[:0], z),
                                       np.float32)
    out["zhjd_empty_out"] = np.array(float(opt.compute_sdf_loss_objectpoint_zhjd(ob.pts[:0], z)))
    meta = {"torch": np.array(torch.__version__), "numpy": np.array(np.__version__)}
    np.savez_compressed(os.path.join(HERE, "f10_edge.npz"), **out, **meta)


if __name__ == "__main__":
    main()
