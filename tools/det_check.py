"""Run-to-run determinism of one small batch per lite-kernel variant (GPU box).

Usage: DSR_LIB=<libdsr.so> python tools/det_check.py [reps]
Prints one hash of (outputs, point counts) per run; every line of a variant must agree.
"""
import ctypes
import hashlib
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)

import synthetic as S  # noqa: E402
from deep_sdf.workspace import decoder_from_state  # noqa: E402
from reconstruct import _libdsr as L  # noqa: E402
import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
lib, ctx = dec.ctx.lib, dec.ctx
os.environ["DSR_LITE"] = "1"
for v, lag in (("88", "4"), ("472", "4"), ("1496", "0"), ("1496", "4")):
    os.environ["DSR_LITE_VARIANT"] = v
    os.environ["DSR_LITE_LAG"] = lag
    for r in range(reps):
        h, keep = bench.make_batch(dec, L.optim_params(S.KITTI_OPTIM), 8, 1000)
        outs = (L.ObjectOut * 8)()
        ctx.check(lib.dsr_batch_run(h), "run")
        ctx.check(lib.dsr_batch_download(h, outs), "download")
        st = L.Stats()
        ctx.check(lib.dsr_batch_stats(h, ctypes.byref(st)), "stats")
        lib.dsr_batch_destroy(h)
        rec = np.array([list(o.t_cam_obj) + list(o.code) + [o.loss, o.is_good, o.iters_done] for o in outs],
                       np.float32)
        hs = hashlib.sha1(rec.tobytes()).hexdigest()[:12]
        print(f"variant {v} lag {lag} rep {r}: {hs} fwd {st.fwd_points} refine {st.refine_points} "
              f"jac {st.jac_points}", flush=True)
