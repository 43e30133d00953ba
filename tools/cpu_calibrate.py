"""Calibrate bench.py's CPU baseline (the numpy oracle port) against the REFERENCE itself,
in the build container:

    python tools/cpu_calibrate.py [--reps 3] [--threads 1,8] > profiles/r4_cpu_calibration.json

Both run the same object — golden F4 ``kitti0`` (KITTI parameters, 2048 surface points,
2048 + 200 rays, 50 depth samples, 10 GN iterations) with the seeded 8x512 decoder — at
the same thread count, each repetition in a fresh child process whose BLAS / OpenMP / torch
intra-op pools are all set to that count:

* ``oracle``: ``oracle.dsr_oracle.reconstruct_object`` (numpy fp32, what bench.py's
  ``cpu_baseline`` leg times on the GPU box);
* ``reference``: the reference's own ``Optimizer.reconstruct_object``
  (/root/reference/reconstruct/optimizer.py:90-205), imported in place through
  tests/golden/refshim.py (torch CPU; never on the GPU box).

The ratio oracle/reference (in obj/s) converts the box's port number into a
reference-equivalent figure (bench.py: ``cpu_baseline.reference_equivalent_value``).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")


def _one(kind):
    import numpy as np

    sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
    sys.path.insert(0, GOLDEN)
    sys.path.insert(0, REPO)
    import synthetic as S

    f = np.load(os.path.join(GOLDEN, "f4_traj_kitti0.npz"), allow_pickle=False)
    T, pts, rays, depth = (np.asarray(f[k], np.float32) for k in
                           ("obj_t_cam_obj", "obj_pts", "obj_rays", "obj_depth"))
    state = S.make_decoder(1234)
    if kind == "oracle":
        from deep_sdf.workspace import fold_state
        from oracle import dsr_oracle as O

        dec = O.Decoder(fold_state(state, S.DEFAULT_SPECS))
        P = O.OptimParams.from_cfg(S.KITTI_OPTIM)
        t0 = time.perf_counter()
        r = O.reconstruct_object(dec, P, T, pts, rays, depth)
        dt = time.perf_counter() - t0
        loss, good = float(r.loss), bool(r.is_good)
    else:
        import torch

        import refshim

        torch.set_num_threads(int(os.environ["DSR_CAL_THREADS"]))
        dec = refshim.build_decoder(state, S.DEFAULT_SPECS)
        opt = refshim.make_optimizer(dec, S.KITTI_OPTIM, "KITTI")
        t0 = time.perf_counter()
        r = opt.reconstruct_object(T.copy(), pts, rays, depth, None)
        dt = time.perf_counter() - t0
        loss, good = float(r.loss), bool(r.is_good)
    print(json.dumps({"seconds": dt, "loss": loss, "is_good": good}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--one", choices=("oracle", "reference"))
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--threads", default=f"1,{os.cpu_count()}")
    a = ap.parse_args()
    if a.one:
        _one(a.one)
        return
    out = {"object": "golden F4 kitti0: KITTI params, 2048 pts, 2248 rays, 50 samples, 10 GN iters",
           "host": {"nproc": os.cpu_count()}, "runs": {}}
    for th in (int(x) for x in a.threads.split(",")):
        env = dict(os.environ, OMP_NUM_THREADS=str(th), OPENBLAS_NUM_THREADS=str(th), MKL_NUM_THREADS=str(th),
                   DSR_CAL_THREADS=str(th), PYTHONDONTWRITEBYTECODE="1")
        for kind in ("oracle", "reference"):
            secs = []
            for _ in range(a.reps):
                p = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", kind], env=env,
                                   capture_output=True, text=True, check=True)
                rec = json.loads(p.stdout.strip().splitlines()[-1])
                secs.append(rec["seconds"])
                print(kind, th, rec, file=sys.stderr, flush=True)
            out["runs"][f"{kind}_{th}t"] = {"seconds": secs, "median_s": statistics.median(secs),
                                            "obj_per_s": 1.0 / statistics.median(secs), "threads": th}
        o, r = out["runs"][f"oracle_{th}t"], out["runs"][f"reference_{th}t"]
        out["runs"][f"port_to_reference_ratio_{th}t"] = o["obj_per_s"] / r["obj_per_s"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
