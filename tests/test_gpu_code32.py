"""CodeLength-32 decoders on the GPU (the reference's C++ caller casts a
32-D code, /root/reference/src/LocalMapping_util.cc:416-422, and deep_sdf_decoder.py:29-56 builds
lin0 35 -> 512, lin3 512 -> 477, lin4 (477 + 35) -> 512 for it).

libdsr runs a 32-D decoder in its 64-D layout: lin0's and lin4's code columns 32..63 are zero,
lin3 has 477 outputs and lin4's GEMM is 480 deep (xyz rows 477..479), the code is held at zero
there.  Its J_code columns 32..63 are then exactly 0, H's code block there is k3 I and its step
0 — the reference's 39-parameter system, solved inside the 71-parameter one.  Checked against
golden F15 (tests/golden/make_code32.py: the reference itself with the seeded 32-D decoder).
"""
from __future__ import annotations

import numpy as np
import pytest

import synthetic as S
from conftest import assert_jac_close, golden, make_cfg

pytestmark = pytest.mark.gpu

SPECS32 = dict(S.DEFAULT_SPECS, CodeLength=32)
KITTI32 = dict(S.KITTI_OPTIM, code_len=32, joint_optim=dict(S.KITTI_OPTIM["joint_optim"], num_iterations=3))


@pytest.fixture(scope="module")
def dec32():
    from deep_sdf.workspace import decoder_from_state

    return decoder_from_state(S.make_decoder(1234, SPECS32), SPECS32)


def _opt(dec, optim):
    from reconstruct.optimizer import Optimizer

    return Optimizer(dec, make_cfg(optim, "KITTI"))


def rel(a, b):
    return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


def test_code32_decoder_vs_golden(dec32):
    from reconstruct.optimizer import sdf_eval

    f = golden("f15_code32.npz")
    assert dec32.code_len == 32 and dec32.info["code_len"] == 32
    y, j = sdf_eval(dec32, f["z"], f["x"], with_jac=True)
    assert j.shape == (256, 35)
    assert np.abs(y - f["sdf"]).max() <= 2e-5
    assert_jac_close(j, f["jac"], tol=1e-4)
    y2 = sdf_eval(dec32, f["z"], f["x"])
    assert np.abs(y2 - f["sdf_nograd"]).max() <= 2e-5
    with pytest.raises(ValueError):
        sdf_eval(dec32, f["z"][:31], f["x"])


def test_code32_teacher_forced_steps(dec32):
    """Every recorded reference state -> one GPU GN step: K, loss, the 39 x 39 H, b and the
    step (H-norm) like the 64-D teacher-forced test; the padded code dimensions exactly inert."""
    f = golden("f15_code32.npz")
    one = dict(KITTI32, joint_optim=dict(KITTI32["joint_optim"], num_iterations=1))
    opt = _opt(dec32, one)
    n_it = int(f["n_iters_run"])
    objs = [(f["it_t_obj_cam"][e], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][e]) for e in range(n_it)]
    res, tr = opt.reconstruct_objects(objs, trace=True, pose_is_obj_cam=True)
    jo = KITTI32["joint_optim"]
    for e in range(n_it):
        t = tr[e]
        assert res[e]["is_good"] and res[e]["code"].shape == (32,)
        dk = abs(int(t["k"][0]) - int(f["it_k"][e]))
        assert dk <= 2
        loss_ref = jo["k1"] * f["it_render_loss"][e] + jo["k2"] * f["it_sdf_loss"][e]
        assert abs(t["loss"][0] - loss_ref) <= 1e-5 * abs(loss_ref) + dk * jo["k1"] * 0.09 / f["it_k"][e]
        H, b, dx = (np.asarray(t[k][0], np.float64) for k in ("H", "b", "dx"))
        # the padded dimensions 39..70: no Jacobian, no right-hand side, no step
        assert (H[39:, :39] == 0).all() and (H[:39, 39:] == 0).all()
        assert np.array_equal(np.diag(H[39:, 39:]), np.full(32, np.float32(jo["k3"]), np.float64))
        assert (H[39:, 39:] == np.diag(np.diag(H[39:, 39:]))).all()
        assert (b[39:] == 0).all() and (dx[39:] == 0).all()
        assert (t["z"][0] == f["it_z"][e]).all()
        eh = rel(H[:39, :39], f["it_H"][e])
        rest = np.r_[0:3, 6:39]
        eb = rel(b[rest], f["it_b"][e][rest])
        d = dx[:39] - f["it_dx"][e]
        Hr = np.asarray(f["it_H"][e], np.float64)
        dr = np.asarray(f["it_dx"][e], np.float64)
        es = float(np.sqrt(max(d @ Hr @ d, 0.0) / max(dr @ Hr @ dr, 1e-300)))
        print(f"code32 it {e}: dK {dk} H {eh:.2e} b {eb:.2e} dx(H-norm) {es:.2e}")
        assert eh <= (5e-4 if dk == 0 else 2e-3)
        assert eb <= (5e-4 if dk == 0 else 5e-3)
        assert es <= 1e-2


def test_code32_trajectory_and_secondary_entry_points(dec32, monkeypatch):
    """The reference's 3-iteration trajectory (same K every iteration up to +-2, loss within the
    teacher-forced bound), a 32-float code back from the Python API on both decode paths, and the
    secondary entry points with a 32-D code: the zhjd query, pose-only GN and mesh extraction."""
    from oracle import dsr_oracle as O
    from reconstruct.optimizer import MeshExtractor

    from deep_sdf.workspace import fold_state

    f = golden("f15_code32.npz")
    opt = _opt(dec32, KITTI32)
    out = {}
    for lite in ("1", "0"):
        monkeypatch.setenv("DSR_LITE", lite)
        (r,), (t,) = opt.reconstruct_objects([(f["obj_t_cam_obj"], f["obj_pts"], f["obj_rays"], f["obj_depth"], None)],
                                             trace=True)
        assert r["is_good"] and r["code"].shape == (32,) and r["iters_done"] == 3
        assert np.abs(t["k"] - f["it_k"]).max() <= 2, (t["k"], f["it_k"])
        out[lite] = r
        print(f"code32 lite={lite}: loss {r['loss']:.6f} (reference {float(f['loss']):.6f}), K {t['k']} / {f['it_k']}")
    assert abs(out["1"]["loss"] - float(f["loss"])) <= 2e-3 * abs(float(f["loss"]))
    r = opt.reconstruct_object(f["obj_t_cam_obj"], f["obj_pts"], f["obj_rays"], f["obj_depth"], out["1"]["code"])
    assert r["is_good"] and r["code"].shape == (32,)
    odec = O.Decoder(fold_state(S.make_decoder(1234, SPECS32), SPECS32), 32, (4,))
    pts_obj = np.random.default_rng(3).uniform(-0.6, 0.6, (500, 3)).astype(np.float32)
    q = opt.compute_sdf_loss_objectpoint_zhjd(pts_obj, out["1"]["code"])
    qo = float(O.compute_sdf_loss_objectpoint(odec, pts_obj, out["1"]["code"]))
    assert abs(q - qo) <= 2e-6
    T = out["1"]["t_cam_obj"].astype(np.float64)
    s = float(np.cbrt(np.linalg.det(T[:3, :3])))
    T_se3 = T.copy()
    T_se3[:3, :3] /= s
    p = opt.estimate_pose_cam_obj(T_se3.astype(np.float32), s, f["obj_pts"], out["1"]["code"])
    po = O.estimate_pose_cam_obj(odec, O.OptimParams.from_cfg(KITTI32), T_se3.astype(np.float32), s, f["obj_pts"],
                                 out["1"]["code"])
    assert np.abs(p - po).max() <= 1e-3 * np.abs(po).max()
    mesh = MeshExtractor(dec32, code_len=32, voxels_dim=32).extract_mesh_from_code(out["1"]["code"])
    assert mesh.vertices.shape[0] > 100 and mesh.faces.shape[0] > 100
