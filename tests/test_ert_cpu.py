"""Early ray termination is exact: the claim behind k_sample_pass, checked on the oracle.

Once a ray sample decodes to sdf <= -th its occupancy is exactly 1 (loss_utils.py:46-47),
the transmittance exactly 0 from there on (loss.py:111), and every later sample of the
ray can only enter the render loss multiplied by an exact zero or be dropped by the
de_do > 1e-2 filter (loss.py:135).  So the outputs of compute_render_loss (loss.py:60-166,
restated in oracle/dsr_oracle.py) must be BITWISE unchanged when the SDF of every sample
behind a ray's first occupied sample is replaced by garbage — which is what the GPU path
does by never decoding those samples.
"""
from __future__ import annotations

import numpy as np
import pytest

import synthetic as S


@pytest.fixture(scope="module")
def setup():
    from deep_sdf.workspace import fold_state
    from oracle import dsr_oracle as O

    dec = O.Decoder(fold_state(S.make_decoder(1234), S.DEFAULT_SPECS))
    P = O.OptimParams.from_cfg(S.KITTI_OPTIM)
    return O, dec, P


@pytest.mark.parametrize("seed,scale,tz", [(11, 2.0, 15.0), (12, 1.0, 3.0)])
def test_render_loss_ignores_samples_behind_termination(setup, seed, scale, tz, monkeypatch):
    O, dec, P = setup
    o = S.make_object(seed, n_pts=160, n_bg=40, scale=scale, tz=tz)
    t_obj_cam = np.linalg.inv(o.t_cam_obj).astype(np.float32)
    s = np.float32(np.cbrt(np.linalg.det(o.t_cam_obj[:3, :3].astype(np.float64))))
    depths = O.linspace_torch(np.float32(o.t_cam_obj[2, 3] - s), np.float32(o.t_cam_obj[2, 3] + s),
                              P.num_depth_samples)
    depth_obs = np.concatenate([o.depth, np.full(o.rays.shape[0] - o.depth.shape[0],
                                                 np.float32(1.1) * depths[-1], np.float32)])
    z = np.zeros(64, np.float32)
    th = P.cut_off
    ref = O.compute_render_loss(dec, o.rays, depth_obs, t_obj_cam, depths, z, th)

    # the in-ball samples in the order compute_render_loss decodes them (loss.py:82)
    obj = O.transform_points(o.rays[:, None, :] * depths[:, None], t_obj_cam)
    vi, _ = np.nonzero(np.sqrt(np.sum(obj * obj, axis=-1)) < 1.0)
    rng = np.random.default_rng(seed)
    true_decode = O.decode_sdf
    skipped = []

    def decode_with_garbage(d, zz, x, max_batch=64 ** 3):
        sdf = true_decode(d, zz, x, max_batch).copy()
        dead = np.zeros(o.rays.shape[0], bool)
        for n in range(sdf.shape[0]):               # (ray, depth) order
            r = vi[n]
            if dead[r]:
                sdf[n] = rng.uniform(-1.0, 1.0)     # never decoded on the GPU
                skipped.append(n)
            elif sdf[n] <= -th:
                dead[r] = True
        return sdf

    monkeypatch.setattr(O, "decode_sdf", decode_with_garbage)
    got = O.compute_render_loss(dec, o.rays, depth_obs, t_obj_cam, depths, z, th)
    assert len(skipped) > 0.1 * vi.shape[0]          # termination does happen here
    assert got.n_valid == ref.n_valid
    for a, b in ((got.j_pose, ref.j_pose), (got.j_code, ref.j_code), (got.res, ref.res),
                 (got.ray_idx, ref.ray_idx), (got.depth_idx, ref.depth_idx), (got.pts, ref.pts)):
        assert np.array_equal(a, b)
