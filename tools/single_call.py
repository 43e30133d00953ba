"""One object per Optimizer.reconstruct_object call — the reference's per-detection pattern
(LocalMapping_util.cc:181-194) — timed back to back (GPU box), for the library DSR_LIB points at;
a hash of every object's result lets two builds be compared for bitwise equality.

Usage: [DSR_LIB=...] python tools/single_call.py [--reps N] [--pts P]
       -> ms per call (median, min) + per-object result hashes
"""
from __future__ import annotations

import argparse
import hashlib
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)

import synthetic as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--pts", type=int, default=2048)
    a = ap.parse_args()
    import ctypes

    from deep_sdf.workspace import decoder_from_state
    from reconstruct import _libdsr as L
    from reconstruct.optimizer import Optimizer
    from reconstruct.utils import ForceKeyErrorDict

    # an A/B against an older build (no trace records are used here): accept its ABI number
    L.ABI_VERSION = ctypes.CDLL(L.lib_path()).dsr_abi_version()

    dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS, device=0)
    opt = Optimizer(dec, ForceKeyErrorDict(data_type="KITTI", optimizer=S.KITTI_OPTIM))
    objs = [S.kitti_object(i, n_pts=a.pts) for i in range(4)]
    opt.reconstruct_object(objs[0].t_cam_obj, objs[0].pts, objs[0].rays, objs[0].depth)
    ts, hashes = [], {}
    for r in range(a.reps):
        o = objs[r % 4]
        t0 = time.perf_counter()
        res = opt.reconstruct_object(o.t_cam_obj, o.pts, o.rays, o.depth)
        ts.append(time.perf_counter() - t0)
        assert res.is_good
        rec = np.concatenate([np.asarray(res.t_cam_obj, np.float32).ravel(), np.asarray(res.code, np.float32).ravel(),
                              np.asarray([res.loss], np.float32)])
        hashes.setdefault(r % 4, set()).add(hashlib.sha1(rec.tobytes()).hexdigest()[:12])
    ts = np.array(ts) * 1e3
    print(f"single reconstruct_object ({a.pts} pts, 10 iters): median {np.median(ts):.3f} ms, "
          f"min {ts.min():.3f} ms over {a.reps} calls", flush=True)
    print("results: " + " ".join(f"obj{i}={','.join(sorted(h))}" for i, h in sorted(hashes.items())), flush=True)


if __name__ == "__main__":
    main()
