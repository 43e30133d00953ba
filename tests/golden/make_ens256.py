"""Golden F13: a 256-member reproducibility ensemble of the REFERENCE on the metric object
(build container only):

    DSR_ENS_JOBS=7 python tests/golden/make_ens256.py [name]      # default: kitti0
    DSR_ENS_THREADS=8 DSR_ENS_JOBS=1 DSR_ENS_MEMBERS=64 python tests/golden/make_ens256.py [name]

The second form is the reference with torch's 8-thread CPU kernels (a different reduction order
from the 1-thread run: SURVEY.md §8(c), K-total 45,584 vs 44,668 on one object) from the first 64
of the same starts -> tests/golden/f18_ens64_t8_<name>.npz: how far the reference's own cloud moves
with its thread count, a second yardstick beside the numpy oracle's (F16).

Each member is the reference's own ``Optimizer.reconstruct_object``
(/root/reference/reconstruct/optimizer.py:90-205; 1 CPU thread, deterministic) on the golden
F4 object (KITTI parameters, 2048 surface points, 2048 + 200 rays, 50 depth samples, 10 GN
iterations) from the fixture's initial pose perturbed by one fp32 ulp (the first 64 members
are ens64's starts, make_ensemble.member_poses).  Recorded per member: the final state and
loss, and per iteration the render-point count K and the two loss terms
(loss.py:22-43 sdf, :60-166 render; the returned loss is k1*render + k2*sdf of the last
pre-update state, optimizer.py:157), so tests/test_gpu_contract.py can compare the GPU's and
the reference's clouds iteration by iteration.  At n = 256 a two-sample KS test at p = 1e-3
rejects a distribution gap of D > ~0.17 (n = 64: ~0.34).

Output: tests/golden/f13_ens256_<name>.npz (t_init, t_cam_obj, code, loss, is_good, it_k,
it_sdf_loss, it_render_loss, plus the generating versions).
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, HERE)

import synthetic as S  # noqa: E402
import refshim  # noqa: E402
import make_golden as MG  # noqa: E402
from make_ensemble import member_poses  # noqa: E402

MEMBERS = int(os.environ.get("DSR_ENS_MEMBERS", "256"))
JOBS = int(os.environ.get("DSR_ENS_JOBS", "7"))
THREADS = int(os.environ.get("DSR_ENS_THREADS", "1"))
_W = {}


def _member(job):
    m, T = job
    f = _W["f"]
    ob = S.SyntheticObject(T.astype(np.float32), f["obj_pts"], f["obj_rays"], f["obj_depth"], None)
    t0 = time.time()
    r, its = MG.run_traj(_W["ref"], _W["dec"], S.KITTI_OPTIM, "KITTI", ob, threads=THREADS)
    n = int(f["n_iters_run"])
    pad = lambda v, fill: list(v) + [fill] * (n - len(v))  # noqa: E731
    print(m, f"{time.time() - t0:.1f}s", float(r.loss), flush=True)
    return (m, np.asarray(r.t_cam_obj if r.is_good else np.full((4, 4), np.nan), np.float32),
            np.asarray(r.code if r.is_good else np.full(64, np.nan), np.float32), float(r.loss), bool(r.is_good),
            pad([i.get("k", -1) for i in its], -1), pad([i.get("sdf_loss", np.nan) for i in its], np.nan),
            pad([i.get("render_loss", np.nan) for i in its], np.nan))


def main():
    import multiprocessing as mp

    import torch

    torch.set_num_threads(THREADS)
    name = ([a for a in sys.argv[1:] if not a.startswith("--")] or ["kitti0"])[0]
    _W["ref"] = refshim.load()
    _W["dec"] = refshim.build_decoder(S.make_decoder(MG.DECODER_SEED), S.DEFAULT_SPECS)
    _W["f"] = dict(np.load(os.path.join(HERE, f"f4_traj_{name}.npz"), allow_pickle=False))
    t_init = member_poses(_W["f"]["obj_t_cam_obj"], MEMBERS)
    jobs = list(enumerate(t_init))
    if JOBS == 1:
        res = [_member(j) for j in jobs]
    else:
        with mp.get_context("fork").Pool(JOBS) as pool:
            res = sorted(pool.map(_member, jobs, chunksize=1), key=lambda r: r[0])
    out = {"t_init": t_init, "t_cam_obj": np.stack([r[1] for r in res]), "code": np.stack([r[2] for r in res]),
           "loss": np.array([r[3] for r in res]), "is_good": np.array([r[4] for r in res]),
           "it_k": np.array([r[5] for r in res], np.int32), "it_sdf_loss": np.array([r[6] for r in res]),
           "it_render_loss": np.array([r[7] for r in res]),
           "torch": np.array(torch.__version__), "numpy": np.array(np.__version__), "threads": np.array(THREADS)}
    fn = f"f13_ens256_{name}.npz" if THREADS == 1 else f"f18_ens{MEMBERS}_t{THREADS}_{name}.npz"
    np.savez_compressed(os.path.join(HERE, fn), **out)


if __name__ == "__main__":
    main()
