"""Extend the F4 trajectory fixtures with a 16-member reproducibility ensemble of the
REFERENCE itself (build container only):

    python tests/golden/make_ensemble.py [name ...]     # default: all four F4 fixtures
    DSR_ENS_MEMBERS=64 DSR_ENS_JOBS=8 python tests/golden/make_ensemble.py   # ens64_*

Each member is the reference's ``reconstruct_object`` (1 CPU thread, deterministic)
from the fixture's initial pose perturbed at the 1e-7 relative level (one fp32 ulp).
The spread of the members' final (t_cam_obj, code, loss) around the unperturbed
1-thread result is how far the reference's own output moves under input rounding —
the envelope tests/test_gpu_contract.py holds the build to on these full-size objects.
Arrays added: ens16_t_cam_obj (16,4,4), ens16_code (16,64), ens16_loss (16,),
ens16_is_good (16,), ens16_k (16, iters), ens16_t_init (16,4,4) (each member's perturbed
initial pose, float32 — what the GPU ensemble of tests/test_gpu_contract.py starts from); with DSR_ENS_MEMBERS=M the same under the
prefix ``ens{M}_`` (the first 16 members get the ens16 perturbations; their results differ
from ens16's in the last bits — the reference's CPU kernels are not reproducible across
processes either), members run in DSR_ENS_JOBS forked 1-thread processes.  The maximum deviation of a
16-member cloud underestimates the cloud's extent; 64 members estimate it better.
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

MEMBERS = int(os.environ.get("DSR_ENS_MEMBERS", "16"))
JOBS = int(os.environ.get("DSR_ENS_JOBS", "1"))
CASES = {"redwood0": (S.REDWOOD_OPTIM, "Redwood"), "redwood1": (S.REDWOOD_OPTIM, "Redwood"),
         "kitti0": (S.KITTI_OPTIM, "KITTI"), "kitti5": (S.KITTI_OPTIM, "KITTI")}
_W = {}


def _member(job):
    """One ensemble member (runs in a worker holding the reference and decoder)."""
    name, m, T = job
    cfg, dtp = CASES[name]
    f = _W["fixtures"][name]
    ob = S.SyntheticObject(T.astype(np.float32), f["obj_pts"], f["obj_rays"], f["obj_depth"], None)
    r, its = MG.run_traj(_W["ref"], _W["dec"], cfg, dtp, ob, threads=1)
    ks = [i.get("k", -1) for i in its]
    print(name, m, float(r.loss), flush=True)
    return (name, m, np.asarray(r.t_cam_obj if r.is_good else np.full((4, 4), np.nan), np.float32),
            np.asarray(r.code if r.is_good else np.full(64, np.nan), np.float32), float(r.loss),
            bool(r.is_good), ks + [-1] * (int(f["n_iters_run"]) - len(ks)))


def member_poses(t_cam_obj, members):
    """The members' perturbed initial poses (float32), in member order."""
    prng = np.random.default_rng(99)
    out = []
    for _ in range(members):
        T = np.asarray(t_cam_obj).astype(np.float64)
        T[:3, :] *= 1.0 + 1e-7 * prng.standard_normal((3, 4))
        out.append(T.astype(np.float32))
    return np.stack(out)


def main():
    import multiprocessing as mp

    import torch

    torch.set_num_threads(1)              # before fork: no intra-op pool in the parent
    names = [a for a in sys.argv[1:] if not a.startswith("--")] or list(CASES)
    if "--init-only" in sys.argv:         # add ens{M}_t_init to fixtures whose members exist
        for name in names:
            path = os.path.join(HERE, f"f4_traj_{name}.npz")
            f = dict(np.load(path, allow_pickle=False))
            f[f"ens{MEMBERS}_t_init"] = member_poses(f["obj_t_cam_obj"], MEMBERS)
            np.savez_compressed(path, **f)
        return
    _W["ref"] = refshim.load()
    _W["dec"] = refshim.build_decoder(S.make_decoder(MG.DECODER_SEED), S.DEFAULT_SPECS)
    _W["fixtures"] = {n: dict(np.load(os.path.join(HERE, f"f4_traj_{n}.npz"), allow_pickle=False))
                      for n in names}
    jobs = []
    for name in names:
        for m, T in enumerate(member_poses(_W["fixtures"][name]["obj_t_cam_obj"], MEMBERS)):
            jobs.append((name, m, T))
    if JOBS > 1:
        with mp.get_context("fork").Pool(JOBS) as pool:
            res = pool.map(_member, jobs, chunksize=1)
    else:
        res = [_member(j) for j in jobs]
    pre = f"ens{MEMBERS}_"
    for name in names:
        rs = sorted((r for r in res if r[0] == name), key=lambda r: r[1])
        f = _W["fixtures"][name]
        f.update({pre + "t_cam_obj": np.stack([r[2] for r in rs]), pre + "code": np.stack([r[3] for r in rs]),
                  pre + "loss": np.array([r[4] for r in rs]), pre + "is_good": np.array([r[5] for r in rs]),
                  pre + "k": np.array([r[6] for r in rs]),
                  pre + "t_init": member_poses(f["obj_t_cam_obj"], MEMBERS)})
        np.savez_compressed(os.path.join(HERE, f"f4_traj_{name}.npz"), **f)


if __name__ == "__main__":
    main()
