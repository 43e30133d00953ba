"""How many ray samples does early ray termination decode under a render-pass schedule?

Offline analysis on the oracle (numpy fp32) along a recorded reference trajectory (F4):
per ray, the in-ball run and the rank of the first sample with sdf <= -th; decoded
samples under (a) the fixed rank windows of k_sample_pass, (b) the minimum (every
sample up to the first full one), (c) windows seeded per ray from the previous
iteration's termination rank (the fixed windows on the first iteration).

Usage: python tools/ert_windows.py [f4 fixture name] [windows...]
"""
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)
import synthetic as S  # noqa: E402
from deep_sdf.workspace import fold_state  # noqa: E402
from oracle import dsr_oracle as O  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "kitti0"
wins = [int(v) for v in sys.argv[2:]] or [0, 8, 12, 16, 20, 24, 32, 50]
f = np.load(os.path.join(REPO, "tests", "golden", f"f4_traj_{name}.npz"))
dec = O.Decoder(fold_state(S.make_decoder(1234), S.DEFAULT_SPECS))
th = 0.01
rays = f["obj_rays"]
prev = None
tot = {"fixed": 0, "min": 0, "pred": 0, "inball": 0}
for e in range(int(f["n_iters_run"])):
    T = f["it_t_obj_cam"][e].astype(np.float32)
    z = f["it_z"][e]
    depths = f["it_depths"][e]
    cam = rays[:, None, :] * depths[:, None]
    obj = O.transform_points(cam, T)
    nrm = np.sqrt((obj * obj).sum(-1))
    inb = nrm < 1.0
    R, M = inb.shape
    sdf = np.full((R, M), np.nan, np.float32)
    vi, vj = np.nonzero(inb)
    sdf[vi, vj] = O.decode_sdf(dec, z, obj[vi, vj])
    cnt = inb.sum(1)
    first = np.argmax(inb, 1)
    # rank (within the in-ball run) of the first full sample, or the run length
    term = np.full(R, -1)
    for r in range(R):
        run = sdf[r, first[r]:first[r] + cnt[r]]
        k = np.nonzero(run <= -th)[0]
        term[r] = k[0] if len(k) else -1
    need = np.where(term >= 0, term + 1, cnt)          # minimum: up to and incl. the first full
    # fixed windows: a ray decodes whole windows until the window holding its first full sample
    fixed = np.zeros(R, int)
    for r in range(R):
        for a, b in zip(wins[:-1], wins[1:]):
            if a >= cnt[r]:
                break
            fixed[r] += min(b, cnt[r]) - a
            if term[r] >= 0 and term[r] < b:
                break
    # predicted: the fixed windows on the first iteration; then a first window [0, p) with
    # p = previous termination + 1 (or the run), then +4 windows
    pred = fixed.copy() if prev is None else np.zeros(R, int)
    for r in range(R if prev is not None else 0):
        p = cnt[r] if prev[r] < 0 else min(cnt[r], prev[r] + 1)
        bnds = [0, p] + list(range(p + 4, cnt[r] + 4, 4))
        for a, b in zip(bnds[:-1], bnds[1:]):
            if a >= cnt[r]:
                break
            pred[r] += min(b, cnt[r]) - a
            if term[r] >= 0 and term[r] < b:
                break
    prev = term
    tot["fixed"] += fixed.sum(); tot["min"] += need.sum(); tot["pred"] += pred.sum(); tot["inball"] += cnt.sum()
    print(f"it {e}: in-ball {cnt.sum()} fixed {fixed.sum()} min {need.sum()} pred {pred.sum()} "
          f"terminated rays {(term >= 0).sum()} of {R}", flush=True)
print({k: int(v) for k, v in tot.items()}, "fixed/min %.3f pred/min %.3f" % (tot["fixed"] / tot["min"], tot["pred"] / tot["min"]))
