"""F12: a 64-member reproducibility ensemble of the REFERENCE at BASELINE config 4's object size
(build container only):

    DSR_ENS_JOBS=6 python tests/golden/make_ens4096.py     # writes tests/golden/f12_ens_kitti4096.npz

The object is f4_traj_kitti4096's (one KITTI object x 4096 surface points x (4096+200) rays), run
at the full KITTI parameter set (10 GN iterations, configs/config_kitti.json) — that fixture holds
a 2-iteration trajectory for teacher forcing.  Recorded: the unperturbed 1-thread result, and 64
members each started from the initial pose perturbed at the 1e-7 relative level (one fp32 ulp;
make_ensemble.member_poses, the same generator as the ens64_ arrays of the F4 fixtures), run
with 1 thread each in forked workers.  tests/test_gpu_contract.py runs the GPU from the same 64
starts and compares the two output clouds (the "distribution" mode of the F4 KITTI objects).
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
from make_ensemble import member_poses  # noqa: E402

MEMBERS = int(os.environ.get("DSR_ENS_MEMBERS", "64"))
JOBS = int(os.environ.get("DSR_ENS_JOBS", "6"))
_W = {}


def _run(job):
    m, T = job
    ob = _W["obj"]
    r, its = MG.run_traj(_W["ref"], _W["dec"], S.KITTI_OPTIM, "KITTI",
                         S.SyntheticObject(T.astype(np.float32), ob.pts, ob.rays, ob.depth, None), threads=1)
    print("member", m, float(r.loss), flush=True)
    return (m, np.asarray(r.t_cam_obj if r.is_good else np.full((4, 4), np.nan), np.float32),
            np.asarray(r.code if r.is_good else np.full(64, np.nan), np.float32), float(r.loss),
            bool(r.is_good), [i.get("k", -1) for i in its])


def main():
    import multiprocessing as mp

    import torch

    torch.set_num_threads(1)
    _W["ref"] = refshim.load()
    _W["dec"] = refshim.build_decoder(S.make_decoder(MG.DECODER_SEED), S.DEFAULT_SPECS)
    ob = S.kitti_object(0, n_pts=4096)
    _W["obj"] = ob
    f4 = np.load(os.path.join(HERE, "f4_traj_kitti4096.npz"), allow_pickle=False)
    assert np.array_equal(f4["obj_pts"], ob.pts) and np.array_equal(f4["obj_rays"], ob.rays)
    jobs = [(-1, ob.t_cam_obj)] + list(enumerate(member_poses(ob.t_cam_obj, MEMBERS)))
    with mp.get_context("fork").Pool(JOBS) as pool:
        res = sorted(pool.map(_run, jobs, chunksize=1), key=lambda r: r[0])
    base, mem = res[0], res[1:]
    n_it = S.KITTI_OPTIM["joint_optim"]["num_iterations"]
    out = dict(obj_t_cam_obj=ob.t_cam_obj, obj_pts=ob.pts, obj_rays=ob.rays, obj_depth=ob.depth,
               num_iterations=np.array(n_it), is_good=np.array(base[4]), t_cam_obj=base[1], code=base[2],
               loss=np.array(base[3], np.float64), it_k=np.array(base[5]),
               ens64_t_cam_obj=np.stack([r[1] for r in mem]), ens64_code=np.stack([r[2] for r in mem]),
               ens64_loss=np.array([r[3] for r in mem]), ens64_is_good=np.array([r[4] for r in mem]),
               ens64_k=np.array([r[5] + [-1] * (n_it - len(r[5])) for r in mem]),
               ens64_t_init=member_poses(ob.t_cam_obj, MEMBERS), torch=np.array(torch.__version__))
    np.savez_compressed(os.path.join(HERE, "f12_ens_kitti4096.npz"), **out)
    print("f12 written: base loss", base[3], "members good", int(sum(r[4] for r in mem)))


if __name__ == "__main__":
    main()
