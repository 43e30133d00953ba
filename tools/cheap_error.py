"""Error of a one-product (hi x hi fp16) decoder pass vs the 3xFP16 pass on realistic samples.

Usage (GPU box): python tools/cheap_error.py
Decodes in-ball ray samples of KITTI-like objects (several shape codes) with fwd variant 12
(3 products) and 140 (hi.hi only) through dsr_sdf_eval and prints the error distribution,
overall and for samples near the occupancy thresholds.
"""
import os, sys
import numpy as np
sys.path.insert(0, "dsp-slam-rgbd_amd"); sys.path.insert(0, ".")
import synthetic as S
from deep_sdf.workspace import decoder_from_state
from reconstruct.optimizer import sdf_eval
from oracle import dsr_oracle as O

dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
P = O.OptimParams.from_cfg(S.KITTI_OPTIM)
errs, vals = [], []
rng = np.random.default_rng(0)
for i in range(6):
    o = S.kitti_object(i, base_seed=1000)
    T = np.linalg.inv(o.t_cam_obj).astype(np.float32)
    s = np.float32(np.cbrt(np.linalg.det(o.t_cam_obj[:3, :3].astype(np.float64))))
    depths = O.linspace_torch(np.float32(o.t_cam_obj[2, 3] - s), np.float32(o.t_cam_obj[2, 3] + s), 50)
    obj = O.transform_points(o.rays[:, None, :] * depths[:, None], T).reshape(-1, 3)
    obj = obj[np.linalg.norm(obj, axis=1) < 1].astype(np.float32)
    for gain in (0.0, 0.3, 1.0):
        code = (gain * rng.standard_normal(64)).astype(np.float32)
        os.environ["DSR_FWD_VARIANT"] = "12"
        a = sdf_eval(dec, code, obj)
        os.environ["DSR_FWD_VARIANT"] = "140"
        b = sdf_eval(dec, code, obj)
        errs.append(np.abs(a - b)); vals.append(a)
e = np.concatenate(errs); v = np.concatenate(vals)
print("samples", e.size, "max err", e.max(), "p99.99", np.percentile(e, 99.99), "p99", np.percentile(e, 99),
      "median", np.median(e))
for lo, hi in ((0, 0.01), (0.01, 0.05), (0.05, 1)):
    m = (np.abs(v) >= lo) & (np.abs(v) < hi)
    print(f"|sdf| in [{lo},{hi}): n={m.sum()} max err {e[m].max() if m.any() else 0:.3g}")
for margin in (0.005, 0.01, 0.02, 0.05):
    refine = np.abs(np.abs(v) - 0.01) < margin + 0.0
    print(f"margin {margin}: refine fraction {(np.abs(v) < 0.01 + margin).mean():.4f}")
