"""test_refine_stops_at_ray_termination's signature under DSR_REFINE_ALL=1 / 0 for the library
DSR_LIB points at (GPU box): record hash, refine / fwd / jac point counts.
Usage: DSR_LIB=... python tools/refine_sig.py"""
import ctypes
import hashlib
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)

import bench  # noqa: E402
import synthetic as S  # noqa: E402
from deep_sdf.workspace import decoder_from_state  # noqa: E402
from reconstruct import _libdsr as L  # noqa: E402

dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
lib, ctx = dec.ctx.lib, dec.ctx
os.environ["DSR_LITE"] = "1"
REPS = int(os.environ.get("REPS", "2"))
MODES = os.environ.get("MODES", "1,0").split(",")
for rep in range(REPS):
    for mode in MODES:
        os.environ["DSR_REFINE_ALL"] = mode
        h, keep = bench.make_batch(dec, L.optim_params(S.KITTI_OPTIM), 8, 1000)
        outs = (L.ObjectOut * 8)()
        ctx.check(lib.dsr_batch_run(h), "run")
        ctx.check(lib.dsr_batch_download(h, outs), "download")
        st = L.Stats()
        ctx.check(lib.dsr_batch_stats(h, ctypes.byref(st)), "stats")
        rec = np.array([list(o.t_cam_obj) + list(o.code) + [o.loss, o.is_good, o.iters_done] for o in outs], np.float32)
        print(f"rep {rep} REFINE_ALL={mode}: rec {hashlib.sha1(rec.tobytes()).hexdigest()[:12]} refine {st.refine_points} "
              f"fwd {st.fwd_points} jac {st.jac_points} viol {st.lite_audit_violations} redo {st.lite_redo_objects} "
              f"maxerr {st.lite_max_err:.3e} broken {st.lite_broken_blocks}", flush=True)
        lib.dsr_batch_destroy(h)
