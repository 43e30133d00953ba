"""hipGraph replay of a keyframe batch (config 5 shape) vs eager, in ONE process per HIP
runtime setting (DEBUG_HIP_FORCE_GRAPH_QUEUES / DEBUG_CLR_GRAPH_PACKET_CAPTURE are read at
HIP init): median ms per re-run and whether the replayed records equal the eager ones.

Usage (GPU box): python tools/graph_queues.py [objects] [reps]
"""
import ctypes as C
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)
import synthetic as S  # noqa: E402
from deep_sdf.workspace import decoder_from_state  # noqa: E402
from reconstruct import _libdsr as L  # noqa: E402

n_obj = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
lib, ctx = dec.ctx.lib, dec.ctx
params = L.optim_params(S.REDWOOD_OPTIM)
keep = []
ins = (L.ObjectIn * n_obj)()
for i in range(n_obj):
    o = S.redwood_object(i)
    arrs = [np.ascontiguousarray(x, np.float32) for x in (o.pts, o.rays, o.depth)]
    keep += arrs
    r = L.ObjectIn()
    r.t_cam_obj[:] = o.t_cam_obj.reshape(-1).tolist()
    r.pts, r.n_pts = L.fptr(arrs[0]), arrs[0].shape[0]
    r.rays, r.n_rays = L.fptr(arrs[1]), arrs[1].shape[0]
    r.depth, r.n_depth = L.fptr(arrs[2]), arrs[2].shape[0]
    ins[i] = r
res = {}
for mode in ("0", "1"):
    os.environ["DSR_GRAPH"] = mode
    h = C.c_void_p()
    ctx.check(lib.dsr_batch_create(ctx.handle, dec.handle, C.byref(params), n_obj, ins, C.byref(h)), "create")
    outs = (L.ObjectOut * n_obj)()
    for _ in range(3):
        ctx.check(lib.dsr_batch_run(h), "run")
        ctx.check(lib.dsr_batch_download(h, outs), "dl")
    t, same = [], True
    first = bytes(outs)
    for _ in range(reps):
        t0 = time.perf_counter()
        ctx.check(lib.dsr_batch_run(h), "run")
        ctx.check(lib.dsr_batch_download(h, outs), "dl")
        t.append(time.perf_counter() - t0)
        same = same and bytes(outs) == first
    lib.dsr_batch_destroy(h)
    res[mode] = (1e3 * float(np.median(t)), first, same)
env = {k: os.environ.get(k, "-") for k in ("DEBUG_HIP_FORCE_GRAPH_QUEUES", "DEBUG_CLR_GRAPH_PACKET_CAPTURE",
                                          "DSR_STREAMS")}
print(f"{env} objects {n_obj}: eager {res['0'][0]:.2f} ms, graph {res['1'][0]:.2f} ms, "
      f"graph records == eager: {res['0'][1] == res['1'][1]}, replays stable: {res['1'][2]}")
