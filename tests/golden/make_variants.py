"""Golden F17: the DeepSDF decoder variants the reference module supports, through the
REFERENCE (build container only; VERDICT r3 "What's missing" 4):

    python tests/golden/make_variants.py

deep_sdf_decoder.py builds, besides the shipped topology, ``use_tanh`` (a tanh after lin8,
before the final ``self.th``, :65-67 / :93-94), ``xyz_in_all`` (every hidden layer but lin3
gives up 3 outputs and every layer input but lin0's / the latent skip's gets xyz appended,
:41-47 / :89-90), plain ``nn.Linear`` layers (weight_norm=False without norm_layers, :49-56) and
LayerNorm layers (weight_norm=False with norm_layers [0..7]: nn.LayerNorm between each lin and
its ReLU, :58-63 / :96-102).
Writes tests/golden/f17_variants.npz, per variant ``<v>_`` (tanh, xyz, plain, ln):
* the seeded decoder (synthetic.make_decoder, seed 1234, the variant's specs) — regenerated
  from the seed by the tests; the SHA-256 of its folded fp32 weights pins it;
* F1-like: sdf (decode_sdf, no grad) and sdf + d sdf / d[code, xyz] (get_batch_sdf_jacobian,
  loss_utils.py:82-113) at 256 points for a random code;
* F4-like (tanh, xyz, ln): Optimizer.reconstruct_object (KITTI parameters, 3 GN iterations, 1 CPU
  thread) on a 512-point KITTI-like object, per-iteration state, H, b, dx, losses and K; and the
  reference's own reproducibility there: 8 starts perturbed by ~1 fp32 ulp (ens8_k, ens8_loss,
  ens8_code).
"""
from __future__ import annotations

import copy
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
from make_ensemble import member_poses  # noqa: E402


def variant_specs(v):
    specs = copy.deepcopy(S.DEFAULT_SPECS)
    ns = specs["NetworkSpecs"]
    if v == "tanh":
        ns["use_tanh"] = True
    elif v == "xyz":
        ns["xyz_in_all"] = True
    elif v == "plain":
        ns["weight_norm"] = False
        ns["norm_layers"] = []
    elif v == "ln":
        ns["weight_norm"] = False            # norm_layers [0..7] of the default specs: LayerNorm
    return specs


VARIANTS = ("tanh", "xyz", "plain", "ln")
KITTI3 = dict(S.KITTI_OPTIM, joint_optim=dict(S.KITTI_OPTIM["joint_optim"], num_iterations=3))


def main():
    import torch

    torch.set_num_threads(1)
    ref = refshim.load()
    out = {"torch": np.array(torch.__version__)}
    for v in VARIANTS:
        specs = variant_specs(v)
        state = S.make_decoder(1234, specs)
        dec = refshim.build_decoder(state, specs)
        h = hashlib.sha256()
        for W, b in MG.folded_layers(dec):
            h.update(W.tobytes())
            h.update(b.tobytes())
        for j in range(8):                       # LayerNorm parameters (variant "ln")
            if hasattr(dec, f"bn{j}"):
                bn = getattr(dec, f"bn{j}")
                h.update(bn.weight.detach().numpy().tobytes())
                h.update(bn.bias.detach().numpy().tobytes())
        out[v + "_folded_sha256"] = np.array(h.hexdigest())
        rng = np.random.default_rng(17)
        z = (0.1 * rng.standard_normal(64)).astype(np.float32)
        x = rng.uniform(-0.9, 0.9, size=(256, 3)).astype(np.float32)
        y, g = ref.loss_utils.get_batch_sdf_jacobian(dec, torch.from_numpy(z), torch.from_numpy(x), 1)
        with torch.no_grad():
            y0 = ref.loss_utils.decode_sdf(dec, torch.from_numpy(z), torch.from_numpy(x))
        out.update({v + "_z": z, v + "_x": x, v + "_sdf": y.detach().numpy().reshape(-1),
                    v + "_jac": g.detach().numpy().reshape(256, 67), v + "_sdf_nograd": y0.numpy().reshape(-1)})
        if v == "plain":
            continue
        ob = S.kitti_object(7, base_seed=1000, n_pts=512)
        r, its = MG.run_traj(ref, dec, KITTI3, "KITTI", ob, threads=1)
        t = MG.pack_traj(r, its)
        out.update({v + "_obj_" + k: a for k, a in (("t_cam_obj", ob.t_cam_obj), ("pts", ob.pts),
                                                    ("rays", ob.rays), ("depth", ob.depth))})
        out.update({v + "_" + k: a for k, a in t.items()})
        print(v, "K per iteration", t["it_k"], "loss", float(r.loss), "is_good", bool(r.is_good))
        # the reference's own reproducibility on this object: 8 starts perturbed by ~1 fp32 ulp
        # (make_ensemble.member_poses), per-iteration K and final loss / code
        ek, el, ez = [], [], []
        for T in member_poses(ob.t_cam_obj, 8):
            ob2 = S.SyntheticObject(T, ob.pts, ob.rays, ob.depth, None)
            r2, its2 = MG.run_traj(ref, dec, KITTI3, "KITTI", ob2, threads=1)
            ek.append([i.get("k", -1) for i in its2])
            el.append(float(r2.loss))
            ez.append(np.asarray(r2.code, np.float32))
        out.update({v + "_ens8_k": np.array(ek), v + "_ens8_loss": np.array(el), v + "_ens8_code": np.stack(ez)})
        print(v, "ens8 K", np.array(ek).min(0), np.array(ek).max(0), "loss", min(el), max(el))
    np.savez_compressed(os.path.join(HERE, "f17_variants.npz"), **out)


if __name__ == "__main__":
    main()
