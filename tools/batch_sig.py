"""Signature of one batch run + one decoder query, for bitwise A/B of two library builds.

Usage (GPU box): DSR_LIB=<path to libdsr.so> python tools/batch_sig.py out.npz
                 python tools/batch_sig.py --compare a.npz b.npz
A layout-only change (LDS swizzles, schedules) must leave every array bitwise equal.
"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8))]
    print("bitwise equal" if not bad else f"DIFFERS: {bad}")
    sys.exit(1 if bad else 0)

import synthetic as S  # noqa: E402
from deep_sdf.workspace import decoder_from_state  # noqa: E402
from reconstruct import _libdsr as L  # noqa: E402

# an A/B against an older build (ABI 10: this script uses only entry points and record layouts
# both ABIs share) — accept the library's own ABI number
L.ABI_VERSION = C.CDLL(L.lib_path()).dsr_abi_version()
from reconstruct.optimizer import sdf_eval  # noqa: E402
import bench  # noqa: E402

dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
lib, ctx = dec.ctx.lib, dec.ctx
n = 16
batch, keep = bench.make_batch(dec, L.optim_params(S.KITTI_OPTIM), n, 1000)
outs = (L.ObjectOut * n)()
ctx.check(lib.dsr_batch_run(batch), "run")
ctx.check(lib.dsr_batch_download(batch, outs), "dl")
st = L.Stats()
ctx.check(lib.dsr_batch_stats(batch, C.byref(st)), "stats")
rec = np.array([list(o.t_cam_obj) + list(o.code) + [o.loss, o.is_good, o.iters_done] for o in outs], np.float32)
cnt = np.array([st.fwd_points, st.refine_points, st.jac_points], np.int64)
rng = np.random.default_rng(0)
z = (0.3 * rng.standard_normal(64)).astype(np.float32)
x = rng.uniform(-0.9, 0.9, (5000, 3)).astype(np.float32)
y, j = sdf_eval(dec, z, x, with_jac=True)
np.savez(sys.argv[1], rec=rec, cnt=cnt, y=y, j=j)
print("saved", sys.argv[1], "loss[0]", rec[0, 80], "pts", cnt)
