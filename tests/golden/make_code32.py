"""Golden F15: a CodeLength-32 DeepSDF decoder through the REFERENCE (build container only;
VERDICT r3 item 7 — the reference's C++ caller has an explicit 32-D branch,
/root/reference/src/LocalMapping_util.cc:416-422, and deep_sdf_decoder.py builds lin0 35 -> 512,
lin3 512 -> 477, lin4 (477 + 35) -> 512 for it):

    python tests/golden/make_code32.py

Writes tests/golden/f15_code32.npz:
* decoder: the seeded 8x512 decoder with CodeLength 32 (synthetic.make_decoder, seed 1234, the
  same generator as the bench decoder) — its state is regenerated from the seed by the tests;
  the SHA-256 of the folded fp32 weights is stored to pin it;
* F1-like: sdf (decode_sdf, no grad) and sdf + d sdf / d[code(32), xyz(3)]
  (get_batch_sdf_jacobian, loss_utils.py:82-113) at 256 points for a random 32-D code;
* F4-like: the reference's Optimizer.reconstruct_object with code_len 32 (KITTI parameters,
  3 GN iterations, 1 CPU thread) on a 512-point KITTI-like object: per-iteration state, H
  (39 x 39), b, dx, losses and K (make_golden.Recorder), and the final result.
"""
from __future__ import annotations

import hashlib
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

SPECS32 = dict(S.DEFAULT_SPECS, CodeLength=32)
KITTI32 = dict(S.KITTI_OPTIM, code_len=32, joint_optim=dict(S.KITTI_OPTIM["joint_optim"], num_iterations=3))


def main():
    import torch

    torch.set_num_threads(1)
    ref = refshim.load()
    state = S.make_decoder(1234, SPECS32)
    dec = refshim.build_decoder(state, SPECS32)
    h = hashlib.sha256()
    for W, b in MG.folded_layers(dec):
        h.update(W.tobytes())
        h.update(b.tobytes())
    out = {"folded_sha256": np.array(h.hexdigest()), "torch": np.array(torch.__version__)}
    rng = np.random.default_rng(32)
    z = (0.1 * rng.standard_normal(32)).astype(np.float32)
    x = rng.uniform(-0.9, 0.9, size=(256, 3)).astype(np.float32)
    y, g = ref.loss_utils.get_batch_sdf_jacobian(dec, torch.from_numpy(z), torch.from_numpy(x), 1)
    with torch.no_grad():
        y0 = ref.loss_utils.decode_sdf(dec, torch.from_numpy(z), torch.from_numpy(x))
    out.update(z=z, x=x, sdf=y.detach().numpy().reshape(-1), jac=g.detach().numpy().reshape(256, 35),
               sdf_nograd=y0.numpy().reshape(-1))
    ob = S.kitti_object(7, base_seed=1000, n_pts=512)
    r, its = MG.run_traj(ref, dec, KITTI32, "KITTI", ob, threads=1)
    t = MG.pack_traj(r, its)
    out.update({"obj_" + k: v for k, v in (("t_cam_obj", ob.t_cam_obj), ("pts", ob.pts), ("rays", ob.rays),
                                             ("depth", ob.depth))})
    out.update(t)
    out["num_iterations"] = np.array(3)
    print("K per iteration", t["it_k"], "loss", float(r.loss), "is_good", bool(r.is_good))
    np.savez_compressed(os.path.join(HERE, "f15_code32.npz"), **out)


if __name__ == "__main__":
    main()
