"""One teacher-forced GN step's terms against fp64 truth, by block (diagnostic, GPU box): from the
recorded reference states of golden F4 (kitti0 / kitti5 / ...), the GPU's H, b and dx (split
kernels as shipped; the fp32-MFMA Jacobian kernel, DSR_JAC_VARIANT=0 under DSR_TEST_HOOKS) and the
reference's own (F4 it_H / it_b / it_dx), each against golden F14 (the numpy oracle in fp64 from
the same state): relative errors of H (pose block, code block), b (translation, rotation, scale,
code) and dx, at identical K.  Usage: python tools/step_probe.py kitti5 [kitti0 ...]"""
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import synthetic as S  # noqa: E402
from conftest import golden, make_cfg  # noqa: E402
from deep_sdf.workspace import decoder_from_state  # noqa: E402
from reconstruct.optimizer import Optimizer  # noqa: E402

dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
BLK = {"b_t": np.s_[0:3], "b_rot": np.s_[3:6], "b_s": np.s_[6:7], "b_code": np.s_[7:71]}


def rel(a, b, sl=np.s_[:]):
    a, b = np.asarray(a, np.float64)[sl], np.asarray(b, np.float64)[sl]
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


for name in sys.argv[1:]:
    f = golden(f"f4_traj_{name}.npz")
    t64 = golden(f"f14_fp64_{name}.npz")
    one = dict(S.KITTI_OPTIM, joint_optim=dict(S.KITTI_OPTIM["joint_optim"], num_iterations=1))
    n_it = min(int(f["n_iters_run"]), 4)
    objs = [(f["it_t_obj_cam"][e], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][e]) for e in range(n_it)]
    runs = {}
    for mode, env in (("split", {}), ("split_jacfwd", {"DSR_TEST_HOOKS": "1", "DSR_SURFACE_EXACT": "0"}),
                      ("jac32", {"DSR_TEST_HOOKS": "1", "DSR_JAC_VARIANT": "0"})):
        for k in ("DSR_TEST_HOOKS", "DSR_JAC_VARIANT", "DSR_SURFACE_EXACT"):
            os.environ.pop(k, None)
        os.environ.update(env)
        opt = Optimizer(dec, make_cfg(one, "KITTI"))
        _, tr = opt.reconstruct_objects(objs, trace=True, pose_is_obj_cam=True)
        runs[mode] = tr
    for e in range(n_it):
        H64, b64, dx64 = (np.asarray(t64[k][e], np.float64) for k in ("H", "b", "dx"))
        line = [f"{name} it {e}: K ref {int(f['it_k'][e])} fp64 {int(t64['k'][e])}"]
        srcs = [("ref", f["it_H"][e], f["it_b"][e], f["it_dx"][e], int(f["it_k"][e]))]
        for mode, tr in runs.items():
            srcs.append((mode, tr[e]["H"][0], tr[e]["b"][0], tr[e]["dx"][0], int(tr[e]["k"][0])))
        for who, H, b, dx, k in srcs:
            Hn = np.asarray(H, np.float64)
            hp, hc = rel(Hn, H64, np.s_[:7, :7]), rel(Hn, H64, np.s_[7:, 7:])
            bb = " ".join(f"{kk} {rel(b, b64, sl):.1e}" for kk, sl in BLK.items())
            dxe = np.asarray(dx, np.float64) - dx64
            hnorm = float(np.sqrt(max(dxe @ H64 @ dxe, 0) / max(dx64 @ H64 @ dx64, 1e-300)))
            line.append(f"  {who:6s} K {k}: H pose {hp:.1e} code {hc:.1e} | {bb} | dx {rel(dx, dx64):.1e} (H-norm {hnorm:.1e})")
        print("\n".join(line), flush=True)
