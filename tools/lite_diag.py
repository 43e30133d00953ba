"""Expired event waits of the staggered lite kernel (k_mlp_fwd_lite_st), read from the device.

Usage (GPU box): python tools/lite_diag.py [reps]
For each (variant, lag, object groups) configuration: run the 8-object KITTI batch `reps`
times and print, per run, the output hash, dsr_stats.lite_broken_blocks and — when a wait
expired — the record of the first one (dsr_batch_lite_diag: workgroup, wave, the counter it
waited on, target vs observed value, tile iteration, HW_ID / XCC_ID, and the real time its
last polls took).  DESIGN.md §3.8 records that variant 216 broke with 2-4 object groups.
"""
import ctypes
import hashlib
import json
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
# (216 needs a -DDSR_LITE_EXPERIMENTS build: DSR_LIB=<that .so> DSR_DIAG_216=1)
configs = [("1496", "4", "4"), ("1496", "0", "4"), ("1496", "4", "2"), ("472", "4", "4")]
if os.environ.get("DSR_DIAG_216") == "1":
    configs += [("216", "0", "4"), ("216", "4", "4"), ("216", "0", "2"), ("216", "0", "1")]
for v, lag, streams in configs:
    os.environ.update(DSR_LITE_VARIANT=v, DSR_LITE_LAG=lag, DSR_STREAMS=streams)
    for r in range(reps):
        h, keep = bench.make_batch(dec, L.optim_params(S.KITTI_OPTIM), 8, 1000)
        try:
            outs = (L.ObjectOut * 8)()
            ctx.check(lib.dsr_batch_run(h), "run")
            ctx.check(lib.dsr_batch_download(h, outs), "download")
            st = L.Stats()
            ctx.check(lib.dsr_batch_stats(h, ctypes.byref(st)), "stats")
            diag = L.lite_diag(lib, h)
        finally:
            lib.dsr_batch_destroy(h)
        rec = np.array([list(o.t_cam_obj) + list(o.code) + [o.loss, o.is_good, o.iters_done] for o in outs],
                       np.float32)
        hs = hashlib.sha1(rec.tobytes()).hexdigest()[:12]
        line = (f"variant {v} lag {lag} streams {streams} rep {r}: {hs} fwd {st.fwd_points} "
                f"refine {st.refine_points} broken_blocks {st.lite_broken_blocks}")
        if diag["recorded"]:
            line += " first_expiry " + json.dumps(diag)
        print(line, flush=True)
