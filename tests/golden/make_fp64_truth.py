"""Golden F14: fp64 "truth" of one GN step from every recorded reference state (build
container):

    python tests/golden/make_fp64_truth.py

For every F4 trajectory fixture and every iteration e, the CPU oracle (oracle/dsr_oracle.py,
pinned to the reference by F1-F8) runs ``gn_step`` in float64 — decoder, sdf / render terms,
rotation prior (/root/reference/reconstruct/loss.py:169-192), damping and the solve
(optimizer.py:161-188) — from the reference's own recorded state (it_t_obj_cam[e], it_z[e]).
The reference's fp32 b and dx at that state (it_b, it_dx) and the GPU's (teacher-forced,
tests/test_gpu_parity.py) are then both measured against the same truth: the GPU must be no
less accurate than the reference itself, in particular on b[3:6], where k4 = 1e7 multiplies an
fp32 cancellation (r_rot = 1 - cos of the tilt).

Output: tests/golden/f14_fp64_<name>.npz with, per iteration, b, dx, H (fp64), K, n_valid and
the loss terms of the fp64 step.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "dsp-slam-rgbd_amd"), REPO]

import synthetic as S  # noqa: E402
from deep_sdf.workspace import fold_state  # noqa: E402
from oracle import dsr_oracle as O  # noqa: E402

CASES = {"redwood0": S.REDWOOD_OPTIM, "redwood1": S.REDWOOD_OPTIM, "kitti0": S.KITTI_OPTIM,
         "kitti5": S.KITTI_OPTIM, "kitti4096": S.KITTI_OPTIM}


def main():
    names = sys.argv[1:] or list(CASES)
    dec = O.Decoder(fold_state(S.make_decoder(1234), S.DEFAULT_SPECS), dtype=np.float64)
    for name in names:
        f = np.load(os.path.join(HERE, f"f4_traj_{name}.npz"), allow_pickle=False)
        P = O.OptimParams.from_cfg(CASES[name])
        pts, rays = f["obj_pts"].astype(np.float64), f["obj_rays"].astype(np.float64)
        depth = f["obj_depth"].astype(np.float64)
        n_fg = depth.shape[0]
        dobs = np.concatenate([depth, np.zeros(rays.shape[0] - n_fg)])
        out = {k: [] for k in ("b", "dx", "H", "k", "n_valid", "loss", "sdf_loss", "render_loss")}
        for e in range(int(f["n_iters_run"])):
            tr, _, _ = O.gn_step(dec, P, f["it_t_obj_cam"][e].astype(np.float64), f["it_z"][e].astype(np.float64),
                                 pts, rays, dobs, n_fg)
            for k in out:
                out[k].append(getattr(tr, k))
            print(name, e, tr.k, int(f["it_k"][e]), flush=True)
        np.savez_compressed(os.path.join(HERE, f"f14_fp64_{name}.npz"),
                            **{k: np.array(v) for k, v in out.items()}, dtype=np.array("float64"))


if __name__ == "__main__":
    main()
