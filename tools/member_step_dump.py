"""One GN step from each of the first members' starts of the 256-member ensemble (golden F13) —
H, b, dx, K, loss — for the shipped split kernels and the fp32-MFMA Jacobian kernel (GPU box),
to compare offline with the fp64 oracle's step from the same starts.
Usage: python tools/member_step_dump.py kitti5 16 -> gpurun_out/member_step_<name>.npz"""
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

name, n = sys.argv[1], int(sys.argv[2])
# optional term isolation: "sdf" (k1 = 0: the render term off) or "render" (k2 = 0)
term = sys.argv[3] if len(sys.argv) > 3 else "both"
KO = dict(S.KITTI_OPTIM["joint_optim"])
if term == "sdf":
    KO["k1"] = 0.0
elif term == "render":
    KO["k2"] = 0.0
dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
f = golden(f"f4_traj_{name}.npz")
e = golden(f"f13_ens256_{name}.npz")
one = dict(S.KITTI_OPTIM, joint_optim=dict(KO, num_iterations=1))
out = {}
for mode, env in (("split", {}), ("jac32", {"DSR_TEST_HOOKS": "1", "DSR_JAC_VARIANT": "0"})):
    for k in ("DSR_TEST_HOOKS", "DSR_JAC_VARIANT"):
        os.environ.pop(k, None)
    os.environ.update(env)
    opt = Optimizer(dec, make_cfg(one, "KITTI"))
    # the members inside a full 256-object batch (the ensemble's launch shapes), first n kept
    objs = [(t, f["obj_pts"], f["obj_rays"], f["obj_depth"], None) for t in e["t_init"]]
    _, tr = opt.reconstruct_objects(objs, trace=True)
    for k in ("H", "b", "dx", "k", "loss", "n_valid"):
        out[f"{mode}_{k}"] = np.array([t[k][0] for t in tr[:n]])
np.savez_compressed(os.path.join(REPO, "gpurun_out", f"member_step_{name}{'' if term == 'both' else '_' + term}.npz"), **out)
print("done")
