"""The north-star output contract (BASELINE.json): final ``t_cam_obj`` / ``code``
within 1e-3 and final ``loss`` within 1e-4 (relative) of the reference's
``Optimizer.reconstruct_object`` (reference optimizer.py:202-205) on identical inputs.

What the reference itself allows: its final outputs are not a
well-conditioned function of its inputs at fp32 precision.  Perturbing only the
initial pose by one fp32 ulp (1e-7 relative) moves the reference's own final code by
up to 4e-1 and its loss by up to 8e-2 on the bench objects (golden F4 ensembles),
because the GN trajectory crosses discontinuous masks (|sdf| = th, de_do = 1e-2,
|x| = 1, the res_rot switch) and every Jacobian point's ReLU kinks.  So the contract
is checked two ways:

* strict, on margin-screened fixtures (F8, tests/golden/make_margin.py): inputs on
  which every iteration keeps every relevant sample >= 1e-5 from each mask threshold
  AND the reference's own 8-member ulp-perturbation ensemble stays within the
  contract (K identical in every member) — there the build must land on the
  reference's result: identical K every
  iteration, final pose (rotation·scale block and translation, max-norm relative) and
  code <= 1e-3, loss <= 1e-4, on both decode paths (DSR_LITE=1 default, DSR_LITE=0);
* by envelope, on the full-size bench objects (F4): the build's deviation from the
  reference's 1-thread result is no larger than twice the largest deviation among the
  members of the reference's own ensemble (64 runs at 1 thread with the initial pose
  perturbed by one fp32 ulp, tests/golden/make_ensemble.py, plus runs at 2/4/8 threads),
  or the contract tolerance where that is larger — i.e. the GPU result is one more member of the reference's own
  reproducibility cloud, for pose, code and loss alike.

The CPU oracle is held to the strict contract on the same F8 fixtures in
``tests/test_oracle_golden.py::test_oracle_final_state_on_margin_fixtures``.
"""
from __future__ import annotations

import glob
import os

import numpy as np
import pytest

import synthetic as S
from conftest import GOLDEN, golden, make_cfg

pytestmark = pytest.mark.gpu

F8 = sorted(glob.glob(os.path.join(GOLDEN, "f8_margin_*.npz")))
POSE_TOL, CODE_TOL, LOSS_TOL = 1e-3, 1e-3, 1e-4


def contract_errors(T, z, loss, f):
    """(rotation-block, translation, code, loss) relative errors vs fixture ``f``."""
    Tr = np.asarray(f["t_cam_obj"], np.float64)
    T = np.asarray(T, np.float64)
    e_rot = np.abs(T[:3, :3] - Tr[:3, :3]).max() / np.abs(Tr[:3, :3]).max()
    e_t = np.abs(T[:3, 3] - Tr[:3, 3]).max() / np.abs(Tr[:3, 3]).max()
    zr = np.asarray(f["code"], np.float64)
    e_z = np.abs(np.asarray(z, np.float64) - zr).max() / np.abs(zr).max()
    e_l = abs(float(loss) - float(f["loss"])) / abs(float(f["loss"]))
    return e_rot, e_t, e_z, e_l


def optim_of(f):
    """The fixture's parameter set (configs/config_kitti.json / config_redwood_01053.json),
    with the iteration count it was generated with."""
    optim, dtp = (S.KITTI_OPTIM, "KITTI") if str(f["data_type"]) == "KITTI" else (S.REDWOOD_OPTIM, "Redwood")
    if "num_iterations" in f.files:
        optim = dict(optim, joint_optim=dict(optim["joint_optim"], num_iterations=int(f["num_iterations"])))
    return optim, dtp


def _run(dec, f, optim, dtp):
    from reconstruct.optimizer import Optimizer

    opt = Optimizer(dec, make_cfg(optim, dtp))
    (r,), (t,) = opt.reconstruct_objects(
        [(f["obj_t_cam_obj"], f["obj_pts"], f["obj_rays"], f["obj_depth"], None)], trace=True)
    return r, t


def test_fixtures_present():
    assert len(F8) >= 2, "margin-screened fixtures missing (python tests/golden/make_margin.py)"


@pytest.mark.parametrize("lite", ["1", "0"])
@pytest.mark.parametrize("path", F8, ids=[os.path.basename(p)[10:-4] for p in F8])
def test_final_state_matches_reference(gpu_decoder, path, lite, monkeypatch):
    monkeypatch.setenv("DSR_LITE", lite)
    f = np.load(path, allow_pickle=False)
    optim, dtp = optim_of(f)
    r, t = _run(gpu_decoder, f, optim, dtp)
    assert r["is_good"] and bool(f["is_good"])
    n_it = int(f["n_iters_run"])
    assert r["iters_done"] == n_it
    assert np.array_equal(t["k"][:n_it], f["it_k"][:n_it]), (t["k"], f["it_k"])
    for e in range(n_it):
        dn = abs(int(t["n_valid"][e]) - int(f["it_n_valid"][e]))
        assert dn == 0 or (dn <= 1 and f["margin_ball_all"][e] < 1e-5), (e, dn)
    e_rot, e_t, e_z, e_l = contract_errors(r["t_cam_obj"], r["code"], r["loss"], f)
    print(f"\n{os.path.basename(path)} lite={lite}: rot {e_rot:.2e} t {e_t:.2e} code {e_z:.2e} "
          f"loss {e_l:.2e} (reference's own spread {f['ref_spread'].tolist()})")
    assert e_rot <= POSE_TOL and e_t <= POSE_TOL, (e_rot, e_t)
    assert e_z <= CODE_TOL, e_z
    assert e_l <= LOSS_TOL, e_l


@pytest.mark.parametrize("path", F8, ids=[os.path.basename(p)[10:-4] for p in F8])
def test_every_iteration_state_tracks_reference(gpu_decoder, path):
    """Not only the end point: every pre-update state (pose, code) of the GPU trajectory
    within the contract's 1e-3 of the reference's state at that iteration, and the loss
    evaluated at it within 1e-3 (intermediate) / 1e-4 (the final one, which is the
    returned ``loss``, optimizer.py:205).  An intermediate loss is taken at the GPU's own
    state, which has drifted from the reference's by up to ~1e-4 (the Jacobian points'
    ReLU kinks move each GN step by ~1e-4), and the loss is not stationary
    before convergence: seen 1.8e-4 at iteration 3 of 5 on redwood_s5359 while its final
    loss agrees to < 1e-4.  From the SAME state the GPU loss agrees to 1e-5
    (test_gpu_parity.py: teacher-forced steps)."""
    f = np.load(path, allow_pickle=False)
    optim, dtp = optim_of(f)
    r, t = _run(gpu_decoder, f, optim, dtp)
    jo = optim["joint_optim"]
    n_it = int(f["n_iters_run"])
    for e in range(n_it):
        Tg, Tr = t["t_obj_cam"][e].astype(np.float64), f["it_t_obj_cam"][e].astype(np.float64)
        e_pose = np.abs(Tg - Tr).max() / np.abs(Tr).max()
        zr = f["it_z"][e].astype(np.float64)
        e_code = np.abs(t["z"][e] - zr).max() / np.abs(zr).max() if np.abs(zr).max() > 0 else 0.0
        loss_ref = jo["k1"] * f["it_render_loss"][e] + jo["k2"] * f["it_sdf_loss"][e]
        e_loss = abs(t["loss"][e] - loss_ref) / abs(loss_ref)
        print(f"it {e}: pose {e_pose:.2e} code {e_code:.2e} loss {e_loss:.2e}")
        assert e_pose <= POSE_TOL and e_code <= CODE_TOL, e
        assert e_loss <= (LOSS_TOL if e == n_it - 1 else POSE_TOL), e


@pytest.mark.parametrize("name,optim,dtp", [("redwood0", S.REDWOOD_OPTIM, "Redwood"),
                                            ("redwood1", S.REDWOOD_OPTIM, "Redwood"),
                                            ("kitti0", S.KITTI_OPTIM, "KITTI"),
                                            ("kitti5", S.KITTI_OPTIM, "KITTI")])
def test_full_size_final_state_within_reference_envelope(gpu_decoder, name, optim, dtp):
    f = golden(f"f4_traj_{name}.npz")
    r, _ = _run(gpu_decoder, f, optim, dtp)
    assert r["is_good"]
    gpu = np.array(contract_errors(r["t_cam_obj"], r["code"], r["loss"], f))
    # every member the fixture holds: 64 (or 16) 1-thread ulp-perturbed runs, plus the 2/4/8
    # thread runs (a perturbation at every reduction, like the GPU's own summation order)
    keys = [k for k in ("ens64_", "ens16_") if k + "loss" in f.files][:1] + ["ens_"]
    ens = np.array([contract_errors(f[k + "t_cam_obj"][m], f[k + "code"][m], f[k + "loss"][m], f)
                    for k in keys for m in range(len(f[k + "loss"]))])
    env = np.nanmax(ens, axis=0)
    tol = np.maximum([POSE_TOL, POSE_TOL, CODE_TOL, LOSS_TOL], 2.0 * env)
    print(f"\n{name}: gpu rot/t/code/loss {np.array2string(gpu, precision=2)} reference ensemble "
          f"{np.array2string(env, precision=2)}")
    assert (gpu <= tol).all(), (gpu, env)
