"""The two 256-member ensemble tests of tests/test_gpu_contract.py, offline, on ensemble dumps
(tools/gpu_ens_dump.py -> gpurun_out/gpu_ens_<tag><object>.npz): how close each kernel variant
comes to every bound (a fraction; > 1 fails), so variants can be ranked from one GPU call that
dumped them all.

  test_ens256_distribution_per_iteration: per-iteration offsets of the loss (reference sigmas)
    and K (render points) from the reference's cloud, against 1.5x the fp32 oracle's largest
    offset + 3 standard errors; final clouds (KS p, printed) and the final-loss mean;
  test_ens_per_iteration_vs_exact_arithmetic: per member against the fp64 oracle (golden F19):
    loss RMS / mean, K bulk (90th percentile of |deviation|), K tails (one-sided Fisher exact
    test), K mean, final states — each against the fp32 implementations' at 1.5x.

usage: python tools/ens_judge.py TAG[,TAG...] [kitti5,kitti0]   (TAG '' = untagged dump)
"""
from __future__ import annotations

import os
import sys

import numpy as np
from scipy.stats import fisher_exact, ks_2samp

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import synthetic as S  # noqa: E402
from conftest import golden  # noqa: E402
from test_gpu_contract import contract_errors  # noqa: E402

JO = S.KITTI_OPTIM["joint_optim"]


def loss_of(g, m=None):
    v = (JO["k1"] * g["it_render_loss"] + JO["k2"] * g["it_sdf_loss"]).astype(np.float64)
    return v if m is None else v[:m]


def judge(name, tag):
    f = golden(f"f4_traj_{name}.npz")
    r, o, x = golden(f"f13_ens256_{name}.npz"), golden(f"f16_oracle_ens256_{name}.npz"), golden(f"f19_oracle64_ens64_{name}.npz")
    g = np.load(os.path.join(REPO, "gpurun_out", f"gpu_ens_{tag}{name}.npz"), allow_pickle=False)
    out = {}

    def worst(k, v):
        out[k] = max(out.get(k, 0.0), float(v))

    # distribution test (all 256 members)
    lr, lo, lg = loss_of(r), loss_of(o), g["it_loss"].astype(np.float64)
    kr, ko, kg = (a["it_k"].astype(np.float64) for a in (r, o, g))
    n, n_it = lr.shape[0], lr.shape[1]
    off_o_l = max(abs(lo[:, e].mean() - lr[:, e].mean()) / lr[:, e].std(ddof=1) for e in range(n_it))
    off_o_k = max(abs(ko[:, e].mean() - kr[:, e].mean()) for e in range(n_it))
    for e in range(n_it):
        sd = lr[:, e].std(ddof=1)
        se = np.sqrt((lg[:, e].var(ddof=1) + lr[:, e].var(ddof=1)) / n) / sd
        worst("dist loss offset", abs(lg[:, e].mean() - lr[:, e].mean()) / sd / (1.5 * off_o_l + 3 * se))
        sek = np.sqrt((kg[:, e].var(ddof=1) + kr[:, e].var(ddof=1)) / n)
        worst("dist K offset", abs(kg[:, e].mean() - kr[:, e].mean()) / (1.5 * off_o_k + 3 * sek))
    g_err = np.array([contract_errors(g["t_cam_obj"][k], g["code"][k], g["loss"][k], f) for k in range(n)])
    r_err = np.array([contract_errors(r["t_cam_obj"][k], r["code"][k], r["loss"][k], f) for k in range(n)])
    out["dist final KS p min"] = min(ks_2samp(g_err[:, k], r_err[:, k]).pvalue for k in range(4))
    gl, rl, ol = (a["loss"].astype(np.float64) for a in (g, r, o))
    se = np.sqrt((gl.var(ddof=1) + rl.var(ddof=1)) / n)
    worst("dist final-loss mean", abs(gl.mean() - rl.mean()) / (1.5 * abs(ol.mean() - rl.mean()) + 3 * se))

    # vs exact arithmetic (first 64 members)
    m = x["it_k"].shape[0]
    lx, lr, lo, lg = loss_of(x, m), loss_of(r, m), loss_of(o, m), lg[:m]
    kx, kr, ko, kg = x["it_k"][:m].astype(np.float64), kr[:m], ko[:m], kg[:m]
    rms = lambda d: float(np.sqrt(np.mean(d * d)))  # noqa: E731
    q90 = lambda d: float(np.quantile(np.abs(d), 0.9))  # noqa: E731
    for e in range(n_it):
        sc = lx[:, e].mean()
        d_g, d_f = (lg[:, e] - lx[:, e]) / sc, [(a[:, e] - lx[:, e]) / sc for a in (lr, lo)]
        worst("exact loss rms", rms(d_g) / (1.5 * max(rms(d) for d in d_f)))
        worst("exact loss mean", abs(d_g.mean()) / (3 * d_g.std(ddof=1) / np.sqrt(m) + 1.5 * max(abs(d.mean()) for d in d_f)))
        k_g, k_f = kg[:, e] - kx[:, e], [a[:, e] - kx[:, e] for a in (kr, ko)]
        q_f = max(q90(d) for d in k_f)
        worst("exact K bulk", q90(k_g) / (1.5 * q_f + 1.0))
        thr = max(3.0, 3.0 * q_f)
        t = lambda d: int((np.abs(d) > thr).sum())  # noqa: E731
        p = min(fisher_exact([[t(k_g), m - t(k_g)], [t(d), m - t(d)]], alternative="greater")[1] for d in k_f)
        worst("exact K tails (1e-3/p)", 1e-3 / max(p, 1e-300))
        worst("exact K mean", abs(k_g.mean()) / (3 * k_g.std(ddof=1) / np.sqrt(m) + 1.5 * max(abs(d.mean()) for d in k_f) + 1e-12))

    def dev(T, z, loss, k):
        T, Tx = np.asarray(T, np.float64), np.asarray(x["t_cam_obj"][k], np.float64)
        zx = np.asarray(x["code"][k], np.float64)
        return (np.abs(T[:3, :3] - Tx[:3, :3]).max() / np.abs(Tx[:3, :3]).max(),
                np.abs(T[:3, 3] - Tx[:3, 3]).max() / np.abs(Tx[:3, 3]).max(),
                np.abs(np.asarray(z, np.float64) - zx).max() / np.abs(zx).max(),
                abs(float(loss) - float(x["loss"][k])) / abs(float(x["loss"][k])))

    fr = lambda a: np.sqrt((np.asarray(a) ** 2).mean(0))  # noqa: E731
    fin_g = fr([dev(g["t_cam_obj"][k], g["code"][k], g["loss"][k], k) for k in range(m)])
    fin_f = np.maximum(*[fr([dev(a["t_cam_obj"][k], a["code"][k], a["loss"][k], k) for k in range(m)]) for a in (r, o)])
    worst("exact final", (fin_g / (1.5 * fin_f)).max())
    return out


def main():
    tags = sys.argv[1].split(",")
    names = (sys.argv[2] if len(sys.argv) > 2 else "kitti5,kitti0").split(",")
    for name in names:
        for tag in tags:
            res = judge(name, tag)
            print(f"{name} {tag or '(untagged)':>10}: " + "  ".join(
                f"{k} {v:.3f}" if "KS" in k else f"{k} {v:.2f}" for k, v in res.items()))


if __name__ == "__main__":
    main()
