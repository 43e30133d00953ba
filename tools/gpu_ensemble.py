"""GPU side of tools/oracle_ensemble.py: the 64 ulp-perturbed initial poses of the reference
ensemble (tests/golden/f4_traj_<name>.npz: ens64_t_init) through libdsr in one batch, per-
iteration K recorded, for each F4 fixture and decode path.  Writes gpurun_out/gpu_ens_<tag>.npz
and prints the K distributions per iteration next to the reference's (ens64_k).

Usage (GPU box): python tools/gpu_ensemble.py <tag> [names...]   (env as for bench.py)
"""
from __future__ import annotations

import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import synthetic as S  # noqa: E402
from deep_sdf.workspace import decoder_from_state  # noqa: E402
from reconstruct.optimizer import Optimizer  # noqa: E402
from reconstruct.utils import ForceKeyErrorDict  # noqa: E402


def main():
    tag = sys.argv[1]
    names = sys.argv[2:] or ["redwood0", "redwood1", "kitti0", "kitti5"]
    dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
    out = {}
    for name in names:
        f = np.load(os.path.join(REPO, "tests", "golden", f"f4_traj_{name}.npz"), allow_pickle=False)
        optim, dtp = (S.KITTI_OPTIM, "KITTI") if name.startswith("kitti") else (S.REDWOOD_OPTIM, "Redwood")
        opt = Optimizer(dec, ForceKeyErrorDict(data_type=dtp, optimizer=optim))
        one = Optimizer(dec, ForceKeyErrorDict(data_type=dtp, optimizer=dict(
            optim, joint_optim=dict(optim["joint_optim"], num_iterations=1))))
        n_it = int(f["n_iters_run"])
        states = [(f["it_t_obj_cam"][e], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][e]) for e in range(n_it)]
        _, ttf = one.reconstruct_objects(states, trace=True, pose_is_obj_cam=True)
        print(f"{name}: teacher-forced K from the reference's states gpu {[int(t['k'][0]) for t in ttf]} "
              f"ref {f['it_k'][:n_it].tolist()}", flush=True)
        for lite in ("1", "0"):
            os.environ["DSR_LITE"] = lite
            res, tr = opt.reconstruct_objects([(f["ens64_t_init"][m], f["obj_pts"], f["obj_rays"], f["obj_depth"],
                                                None) for m in range(64)], trace=True)
            key = f"{name}_lite{lite}"
            out[key + "_t_cam_obj"] = np.stack([np.asarray(r["t_cam_obj"], np.float32) for r in res])
            out[key + "_code"] = np.stack([np.asarray(r["code"], np.float32) for r in res])
            out[key + "_loss"] = np.array([r["loss"] for r in res])
            out[key + "_k"] = np.stack([t["k"] for t in tr])
            print(f"{key}: loss mean {out[key + '_loss'].mean():.6f} (ref {f['ens64_loss'].mean():.6f})", flush=True)
            for it in range(out[key + "_k"].shape[1]):
                ug, cg = np.unique(out[key + "_k"][:, it], return_counts=True)
                ur, cr = np.unique(f["ens64_k"][:, it], return_counts=True)
                print(f"  K it {it}: gpu {dict(zip(ug.tolist(), cg.tolist()))} ref {dict(zip(ur.tolist(), cr.tolist()))}",
                      flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(REPO, "gpurun_out", f"gpu_ens_{tag}.npz"), **out)


if __name__ == "__main__":
    main()
