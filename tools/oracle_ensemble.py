"""The CPU oracle (numpy fp32, oracle/dsr_oracle.py) from the reference ensemble's 64 ulp-
perturbed initial poses (tests/golden/f4_traj_<name>.npz: ens64_t_init), compared with the
reference's own ensemble the way tests/test_gpu_contract.py compares the GPU's: a third
fp32 implementation of the same algorithm, to tell an implementation bug from the
reference's sensitivity to rounding at a near-threshold sample.

Usage: python tools/oracle_ensemble.py redwood0 [jobs]   (CPU; writes /tmp/oracle_ens_<name>.npz)
"""
from __future__ import annotations

import multiprocessing as mp
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import synthetic as S  # noqa: E402

_W = {}


def _init(name):
    from deep_sdf.workspace import fold_state
    from oracle import dsr_oracle as O

    f = dict(np.load(os.path.join(REPO, "tests", "golden", f"f4_traj_{name}.npz"), allow_pickle=False))
    optim = S.KITTI_OPTIM if name.startswith("kitti") else S.REDWOOD_OPTIM
    _W.update(O=O, f=f, dec=O.Decoder(fold_state(S.make_decoder(1234), S.DEFAULT_SPECS)),
              P=O.OptimParams.from_cfg(optim))


def _member(m):
    f, O = _W["f"], _W["O"]
    r = O.reconstruct_object(_W["dec"], _W["P"], f["ens64_t_init"][m], f["obj_pts"], f["obj_rays"], f["obj_depth"])
    return (np.asarray(r.t_cam_obj, np.float32), np.asarray(r.code, np.float32), float(r.loss), bool(r.is_good),
            [t.k for t in r.trace])


def main():
    name = sys.argv[1]
    jobs = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    with mp.get_context("fork").Pool(jobs, initializer=_init, initargs=(name,)) as pool:
        res = pool.map(_member, range(64), chunksize=1)
    T = np.stack([r[0] for r in res])
    z = np.stack([r[1] for r in res])
    loss = np.array([r[2] for r in res])
    ks = np.array([r[4] for r in res])
    np.savez(f"/tmp/oracle_ens_{name}.npz", t_cam_obj=T, code=z, loss=loss, k=ks)
    from test_gpu_contract import contract_errors

    f = np.load(os.path.join(REPO, "tests", "golden", f"f4_traj_{name}.npz"), allow_pickle=False)
    o_err = np.array([contract_errors(T[m], z[m], loss[m], f) for m in range(64)])
    r_err = np.array([contract_errors(f["ens64_t_cam_obj"][m], f["ens64_code"][m], f["ens64_loss"][m], f)
                      for m in range(64)])
    from scipy.stats import ks_2samp

    rl = f["ens64_loss"]
    se = np.sqrt((rl.var(ddof=1) + loss.var(ddof=1)) / 64)
    print(f"{name}: loss mean oracle {loss.mean():.6f} ref {rl.mean():.6f} |d| {abs(loss.mean() - rl.mean()):.2e} "
          f"3 SE {3 * se:.2e}; KS p {ks_2samp(loss, rl).pvalue:.3f}")
    for k, c in enumerate(("rot", "t", "code")):
        print(f"  {c}: median oracle {np.median(o_err[:, k]):.2e} ref {np.median(r_err[:, k]):.2e} "
              f"KS p {ks_2samp(o_err[:, k], r_err[:, k]).pvalue:.3f}")
    for it in range(ks.shape[1]):
        uo, co = np.unique(ks[:, it], return_counts=True)
        ur, cr = np.unique(f["ens64_k"][:, it], return_counts=True)
        print(f"  K it {it}: oracle {dict(zip(uo.tolist(), co.tolist()))} ref {dict(zip(ur.tolist(), cr.tolist()))}")


if __name__ == "__main__":
    main()
