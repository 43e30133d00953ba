"""Accuracy probe (GPU; diagnostic, not a test): where does the GPU's b / dx error vs the fp64
truth come from, and how do the 256-member ensemble clouds compare per iteration.

    python tools/acc_probe.py [split,fp32,split_nolite] > gpurun_out/acc_probe.json

Part 1 — from every recorded reference state of golden F4 (teacher forced, one GN step), the
error of b[3:6], b[rest] and dx vs golden F14 (fp64 oracle) for the shipped decode (split-fp16
MFMA, DSR_FWD_VARIANT / DSR_JAC_VARIANT 12) and for the fp32-MFMA kernels (variants 0), next to
the reference's own fp32 error.  Part 2 — per iteration of the F13 ensemble (kitti0, 256
ulp-perturbed starts): K and loss means, spreads and KS p-values, GPU vs reference.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))

from conftest import golden, make_cfg  # noqa: E402
import synthetic as S  # noqa: E402


def errs(tr, f, t64, n_it):
    out = {"b_rot": [], "b_rest": [], "dx": []}
    for e in range(n_it):
        if not (int(tr[e]["k"][0]) == int(f["it_k"][e]) == int(t64["k"][e])):
            continue
        b64, dx64 = np.asarray(t64["b"][e], np.float64), np.asarray(t64["dx"][e], np.float64)
        for key, sl in (("b_rot", np.s_[3:6]), ("b_rest", np.r_[0:3, 6:71])):
            sc = np.abs(b64[sl]).max()
            out[key].append([float(np.abs(np.asarray(tr[e]["b"][0], np.float64)[sl] - b64[sl]).max() / sc),
                             float(np.abs(np.asarray(f["it_b"][e], np.float64)[sl] - b64[sl]).max() / sc)])
        sc = np.abs(dx64).max()
        out["dx"].append([float(np.abs(np.asarray(tr[e]["dx"][0], np.float64) - dx64).max() / sc),
                          float(np.abs(np.asarray(f["it_dx"][e], np.float64) - dx64).max() / sc)])
    return out


def main():
    from deep_sdf.workspace import decoder_from_state
    from reconstruct.optimizer import Optimizer
    from scipy.stats import ks_2samp

    dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
    rep = {"teacher_forced": {}, "ens256": []}
    cases = [("redwood0", S.REDWOOD_OPTIM, "Redwood"), ("redwood1", S.REDWOOD_OPTIM, "Redwood"),
             ("kitti0", S.KITTI_OPTIM, "KITTI"), ("kitti5", S.KITTI_OPTIM, "KITTI")]
    modes = (("split", {}), ("fp32", {"DSR_FWD_VARIANT": "0", "DSR_JAC_VARIANT": "0"}),
             ("split_nolite", {"DSR_LITE": "0"}))
    want = sys.argv[1].split(",") if len(sys.argv) > 1 else [m for m, _ in modes]
    for mode, env in modes:
        if mode not in want:
            continue
        for k in ("DSR_FWD_VARIANT", "DSR_JAC_VARIANT", "DSR_LITE"):
            os.environ.pop(k, None)
        os.environ.update(env)
        for name, optim, dtype in cases:
            f = golden(f"f4_traj_{name}.npz")
            t64 = golden(f"f14_fp64_{name}.npz")
            one = dict(optim, joint_optim=dict(optim["joint_optim"], num_iterations=1))
            opt = Optimizer(dec, make_cfg(one, dtype))
            n_it = int(f["n_iters_run"])
            objs = [(f["it_t_obj_cam"][e], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][e])
                    for e in range(n_it)]
            _, tr = opt.reconstruct_objects(objs, trace=True, pose_is_obj_cam=True)
            r = errs(tr, f, t64, n_it)
            summ = {k: {"gpu_rms": float(np.sqrt((np.array(v)[:, 0] ** 2).mean())),
                        "ref_rms": float(np.sqrt((np.array(v)[:, 1] ** 2).mean())),
                        "gpu_med": float(np.median(np.array(v)[:, 0])),
                        "ref_med": float(np.median(np.array(v)[:, 1])), "per_it": v} for k, v in r.items()}
            rep["teacher_forced"][f"{mode}/{name}"] = summ
            print(mode, name, {k: (f"{s['gpu_rms']:.2e}/{s['ref_rms']:.2e}", f"{s['gpu_med']:.2e}/{s['ref_med']:.2e}")
                               for k, s in summ.items()}, file=sys.stderr, flush=True)
    for k in ("DSR_FWD_VARIANT", "DSR_JAC_VARIANT", "DSR_LITE"):
        os.environ.pop(k, None)
    f = golden("f4_traj_kitti0.npz")
    e256 = golden("f13_ens256_kitti0.npz")
    n = e256["t_init"].shape[0]
    opt = Optimizer(dec, make_cfg(S.KITTI_OPTIM, "KITTI"))
    _, tr = opt.reconstruct_objects([(e256["t_init"][m], f["obj_pts"], f["obj_rays"], f["obj_depth"], None)
                                     for m in range(n)], trace=True)
    jo = S.KITTI_OPTIM["joint_optim"]
    rep["ens_gpu_k"] = [[int(x) for x in t["k"]] for t in tr]
    rep["ens_gpu_loss"] = [[float(x) for x in t["loss"]] for t in tr]
    for e in range(int(f["n_iters_run"])):
        kg = np.array([t["k"][e] for t in tr], np.float64)
        kr = e256["it_k"][:, e].astype(np.float64)
        lg = np.array([t["loss"][e] for t in tr], np.float64)
        lr = jo["k1"] * e256["it_render_loss"][:, e] + jo["k2"] * e256["it_sdf_loss"][:, e]
        row = {"it": e, "k_mean": [kg.mean(), kr.mean()], "k_std": [kg.std(ddof=1), kr.std(ddof=1)],
               "k_ks": float(ks_2samp(kg, kr).pvalue), "k_hist_gpu": np.unique(kg, return_counts=True)[1].tolist()[:8],
               "loss_mean": [lg.mean(), lr.mean()], "loss_std": [lg.std(ddof=1), lr.std(ddof=1)],
               "loss_ks": float(ks_2samp(lg, lr).pvalue),
               "k_values": [np.unique(kg).tolist()[:8], np.unique(kr).tolist()[:8]]}
        rep["ens256"].append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    print(json.dumps(rep))


if __name__ == "__main__":
    main()
