"""One KITTI object per ``Optimizer.reconstruct_object`` call (BASELINE configs[1], bench.py's
config1_single) for the library DSR_LIB points at (GPU box): ms per call over N calls and a hash
of the result, so two builds can be compared for speed and bitwise equality.
Usage: DSR_LIB=... python tools/single_call.py [N]"""
import hashlib
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)

import synthetic as S  # noqa: E402
from deep_sdf.workspace import decoder_from_state  # noqa: E402
from reconstruct.optimizer import Optimizer  # noqa: E402
from reconstruct.utils import ForceKeyErrorDict  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS, device=0)
opt = Optimizer(dec, ForceKeyErrorDict(data_type="KITTI", optimizer=S.KITTI_OPTIM))
for i in range(3):
    o = S.kitti_object(i, base_seed=1000, n_pts=2048)
    args = (o.t_cam_obj, o.pts, o.rays, o.depth)
    r = opt.reconstruct_object(*args)                        # warm-up
    t0 = time.perf_counter()
    for _ in range(n):
        r = opt.reconstruct_object(*args)
    ms = (time.perf_counter() - t0) / n * 1e3
    rec = np.concatenate([np.asarray(r.t_cam_obj, np.float32).ravel(), np.asarray(r.code, np.float32).ravel(),
                          np.asarray([r.loss, r.is_good], np.float32)])
    print(f"object {i}: {ms:.3f} ms per call, result {hashlib.sha1(rec.tobytes()).hexdigest()[:12]}", flush=True)
