"""Extend the F4 trajectory fixtures with a 16-member reproducibility ensemble of the
REFERENCE itself (build container only):

    python tests/golden/make_ensemble.py [name ...]     # default: all four F4 fixtures

Each member is the reference's ``reconstruct_object`` (1 CPU thread, deterministic)
from the fixture's initial pose perturbed at the 1e-7 relative level (one fp32 ulp).
The spread of the members' final (t_cam_obj, code, loss) around the unperturbed
1-thread result is how far the reference's own output moves under input rounding —
the envelope tests/test_gpu_contract.py holds the build to on these full-size objects.
Arrays added: ens16_t_cam_obj (16,4,4), ens16_code (16,64), ens16_loss (16,),
ens16_is_good (16,), ens16_k (16, iters).
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

MEMBERS = 16
CASES = {"redwood0": (S.REDWOOD_OPTIM, "Redwood"), "redwood1": (S.REDWOOD_OPTIM, "Redwood"),
         "kitti0": (S.KITTI_OPTIM, "KITTI"), "kitti5": (S.KITTI_OPTIM, "KITTI")}


def main():
    names = sys.argv[1:] or list(CASES)
    ref = refshim.load()
    dec = refshim.build_decoder(S.make_decoder(MG.DECODER_SEED), S.DEFAULT_SPECS)
    for name in names:
        cfg, dtp = CASES[name]
        path = os.path.join(HERE, f"f4_traj_{name}.npz")
        f = dict(np.load(path, allow_pickle=False))
        prng = np.random.default_rng(99)
        T_, z_, l_, g_, k_ = [], [], [], [], []
        for m in range(MEMBERS):
            T = f["obj_t_cam_obj"].astype(np.float64)
            T[:3, :] *= 1.0 + 1e-7 * prng.standard_normal((3, 4))
            ob = S.SyntheticObject(T.astype(np.float32), f["obj_pts"], f["obj_rays"], f["obj_depth"], None)
            r, its = MG.run_traj(ref, dec, cfg, dtp, ob, threads=1)
            T_.append(np.asarray(r.t_cam_obj if r.is_good else np.full((4, 4), np.nan), np.float32))
            z_.append(np.asarray(r.code if r.is_good else np.full(64, np.nan), np.float32))
            l_.append(float(r.loss))
            g_.append(bool(r.is_good))
            ks = [i.get("k", -1) for i in its]
            k_.append(ks + [-1] * (int(f["n_iters_run"]) - len(ks)))
            print(name, m, float(r.loss), flush=True)
        f.update(ens16_t_cam_obj=np.stack(T_), ens16_code=np.stack(z_), ens16_loss=np.array(l_),
                 ens16_is_good=np.array(g_), ens16_k=np.array(k_))
        np.savez_compressed(path, **f)


if __name__ == "__main__":
    main()
