"""A/B kernel variants (an env switch: DSR_LITE_VARIANT, DSR_SPLIT_RING, ...) in ONE process,
interleaved.

Usage (GPU box): python tools/lite_variants.py 16 24 [--var DSR_LITE_VARIANT | DSR_RENDER_PASSES ...] [--diag 18] [--rounds 5] [--iters 1]
Each run is a batch of `--iters` GN iterations over 64 KITTI-like objects.  Prints the median
lite-kernel ms per launch and TFLOP/s (one fp16 product per MAC), and checks that every
non-diagnostic variant returns results bitwise equal to the first one (the variants only change
the schedule, never the k order of any accumulation).  `--diag` variants are timing experiments
with invalid results (dsr_api.hip: lite_kernel) and are not compared.
"""
import argparse
import ctypes as C
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

ap = argparse.ArgumentParser()
ap.add_argument("variants", nargs="*", default=["0"])
ap.add_argument("--diag", nargs="*", default=[])
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--objects", type=int, default=64)
ap.add_argument("--iters", type=int, default=1)
ap.add_argument("--var", default="DSR_LITE_VARIANT")
a = ap.parse_args()
dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
cfg = dict(S.KITTI_OPTIM, joint_optim=dict(S.KITTI_OPTIM["joint_optim"], num_iterations=a.iters))
lib, ctx = dec.ctx.lib, dec.ctx
outs = (L.ObjectOut * a.objects)()
allv = list(a.variants) + list(a.diag)
res = {v: [] for v in allv}
batches = {}
for v in allv:     # one batch per variant: switches read at batch creation (DSR_RENDER_PASSES) apply too
    os.environ[a.var] = str(v)
    batches[v] = bench.make_batch(dec, L.optim_params(cfg), a.objects, 1000)
ref = None
bad = []
for r in range(a.rounds):
    for v in allv:
        os.environ[a.var] = str(v)
        batch = batches[v][0]
        ctx.check(lib.dsr_batch_run(batch), "run")
        ctx.check(lib.dsr_batch_download(batch, outs), "dl")
        st = L.Stats()
        ctx.check(lib.dsr_batch_stats(batch, C.byref(st)), "stats")
        res[v].append((st.fwd_ms / max(1, st.fwd_launches), st.fwd_ms, st.total_ms,
                       2 * bench.FWD_MAC * st.fwd_points / (st.fwd_ms * 1e-3) / 1e12, st.fwd_points,
                       st.refine_ms, st.jac_ms, st.refine_points))
        if v in a.variants:
            sig = np.array([list(outs[i].t_cam_obj) + list(outs[i].code) + [outs[i].loss]
                            for i in range(a.objects)], np.float32)
            if ref is None:
                ref = sig
            elif not np.array_equal(sig.view(np.uint32), ref.view(np.uint32)) and v not in bad:
                bad.append(v)
for v in allv:
    x = np.median(np.array(res[v]), axis=0)
    tag = "diag" if v in a.diag else ("DIFFERS" if v in bad else "bitwise-equal")
    print(f"{a.var}={v}: lite {x[0]:6.3f} ms/launch {x[1]:7.2f} ms/run {x[3]:7.1f} TF | exact band "
          f"{x[5]:6.2f} ms | jac {x[6]:6.2f} ms | total {x[2]:7.2f} ms | pts {int(x[4])} refine {int(x[7])}  [{tag}]", flush=True)
if bad:
    sys.exit(1)
