"""Config 5 shape (BASELINE.json): per-keyframe batches of 8 Redwood-parameter objects
(512 pts, 712 rays, 5 GN iters) re-run back to back, eager vs hipGraph replay.

Usage (GPU box): python tools/keyframe_bench.py [--objects 8] [--reps 20]
"""
import argparse, os, sys, time
import numpy as np
REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd")); sys.path.insert(0, REPO)
import synthetic as S
from deep_sdf.workspace import decoder_from_state
from reconstruct import _libdsr as L
from reconstruct.optimizer import Optimizer
from reconstruct.utils import ForceKeyErrorDict

ap = argparse.ArgumentParser()
ap.add_argument("--objects", type=int, default=8)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
lib, ctx = dec.ctx.lib, dec.ctx
params = L.optim_params(S.REDWOOD_OPTIM)
objs = [S.redwood_object(i) for i in range(a.objects)]
ins = (L.ObjectIn * a.objects)()
keep = []
for i, o in enumerate(objs):
    arrs = [np.ascontiguousarray(x, np.float32) for x in (o.pts, o.rays, o.depth)]
    keep += arrs
    r = L.ObjectIn()
    r.t_cam_obj[:] = o.t_cam_obj.reshape(-1).tolist()
    r.pts, r.n_pts = L.fptr(arrs[0]), arrs[0].shape[0]
    r.rays, r.n_rays = L.fptr(arrs[1]), arrs[1].shape[0]
    r.depth, r.n_depth = L.fptr(arrs[2]), arrs[2].shape[0]
    r.code = None
    ins[i] = r
import ctypes as C
outs = (L.ObjectOut * a.objects)()
for mode in ("0", "1"):
    os.environ["DSR_GRAPH"] = mode
    h = C.c_void_p()
    ctx.check(lib.dsr_batch_create(ctx.handle, dec.handle, C.byref(params), a.objects, ins, C.byref(h)), "create")
    for _ in range(3):
        ctx.check(lib.dsr_batch_run(h), "run"); ctx.check(lib.dsr_batch_download(h, outs), "dl")
    t = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        ctx.check(lib.dsr_batch_run(h), "run"); ctx.check(lib.dsr_batch_download(h, outs), "dl")
        t.append(time.perf_counter() - t0)
    lib.dsr_batch_destroy(h)
    good = sum(outs[i].is_good for i in range(a.objects))
    print(f"graph={mode}: keyframe batch of {a.objects} objects: median {1e3*np.median(t):.2f} ms "
          f"(min {1e3*min(t):.2f}) -> {a.objects/np.median(t):.1f} obj/s, good {good}/{a.objects}")
# the reference's call pattern: one reconstruct_object per detection (LocalMapping_util.cc:165-206)
t = []
for _ in range(max(3, a.reps // 4)):
    t0 = time.perf_counter()
    for i in range(a.objects):
        o1 = (L.ObjectOut * 1)()
        ctx.check(lib.dsr_reconstruct_batch(ctx.handle, dec.handle, C.byref(params), 1, C.byref(ins[i]), o1, None),
                  "one")
    t.append(time.perf_counter() - t0)
print(f"one call per object: {a.objects} objects: median {1e3*np.median(t):.2f} ms -> "
      f"{a.objects/np.median(t):.1f} obj/s")
