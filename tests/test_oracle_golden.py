"""Pin the CPU oracle (oracle/dsr_oracle.py) to the reference's golden vectors.

The fixtures were produced by the reference's own Python (tests/golden/make_golden.py,
build container only).  These tests run on CPU and gate the oracle before it is
trusted as the checker of the HIP path.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

import synthetic as S
from conftest import assert_jac_close, golden
from oracle import dsr_oracle as O


def rel(a, b):
    return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


def test_fixture_decoder_is_the_generated_one(full_state):
    g = golden("f0_fold.npz")
    assert str(g["full_state_sha256"]) == S.state_sha256(full_state)


def test_weight_norm_fold_bit_exact(full_layers):
    """deep_sdf.workspace.fold_state (used by the product loader) == the reference
    module's weight-norm hook, bit for bit (F0)."""
    import hashlib

    from deep_sdf.workspace import fold_state
    from tests.golden.make_golden import SMALL_SPECS

    g = golden("f0_fold.npz")
    h = hashlib.sha256()
    for W, b in full_layers:
        h.update(W.tobytes())
        h.update(b.tobytes())
    assert h.hexdigest() == str(g["full_folded_sha256"])
    import re

    state = {}
    for k in g.files:
        m = re.match(r"state_module_lin(\d+)_(weight_g|weight_v|weight|bias)$", k)
        if m:
            state[f"module.lin{m.group(1)}.{m.group(2)}"] = g[k]
    small = fold_state(state, SMALL_SPECS)
    for i, (W, b) in enumerate(small):
        assert np.array_equal(W, g[f"W{i}"]) and np.array_equal(b, g[f"b{i}"])


@pytest.mark.parametrize("name", ["small", "full"])
def test_decoder_fwd_jac(name):
    from deep_sdf.workspace import fold_state
    from tests.golden.make_golden import SMALL_SEED, SMALL_SPECS

    g = golden(f"f1_decoder_{name}.npz")
    if name == "small":
        layers = fold_state(S.make_decoder(SMALL_SEED, SMALL_SPECS), SMALL_SPECS)
        dec = O.Decoder(layers, 16, (4,))
    else:
        layers = fold_state(S.make_decoder(1234), S.DEFAULT_SPECS)
        dec = O.Decoder(layers, 64, (4,))
    L = g["z"].shape[0]
    inp = np.concatenate([np.broadcast_to(g["z"], (g["x"].shape[0], L)), g["x"]], 1)
    y, j = dec.forward_jac(inp)
    assert np.abs(y - g["sdf"]).max() <= 2e-5
    assert_jac_close(j, g["jac"])
    assert np.abs(O.decode_sdf(dec, g["z"], g["x"]) - g["sdf_nograd"]).max() <= 2e-5


def test_sdf_and_render_terms(oracle_dec):
    """F2/F3: compute_sdf_loss / compute_render_loss at one state."""
    f = golden("f23_terms.npz")
    ob = S.redwood_object(0)
    T, z = f["t_obj_cam"], f["z"]
    jp, jc, r = O.compute_sdf_loss(oracle_dec, ob.pts, T, z)
    assert np.abs(r - f["sdf_res"]).max() <= 2e-5
    assert rel(jp, f["sdf_j_pose"]) <= 2e-5 and rel(jc, f["sdf_j_code"]) <= 2e-5
    ren = O.compute_render_loss(oracle_dec, ob.rays, f["depth_obs"], T, f["depths"], z, 0.01)
    # the sampled points are bit-exact (same fp32 op order as the reference)
    assert np.array_equal(np.stack([ren.pts]), np.stack([f["render_pts"]]))
    assert ren.n_valid == f["render_query"].shape[0]
    assert ren.res.shape == f["render_res"].shape
    assert np.abs(ren.res - f["render_res"]).max() <= 5e-5
    assert rel(ren.j_pose, f["render_j_pose"]) <= 5e-4
    assert rel(ren.j_code, f["render_j_code"]) <= 5e-4


def test_linspace_and_small_math():
    """F5: torch.linspace (fp32 CPU), exp_sim3 / exp_se3, Huber, rotation prior."""
    f = golden("f5_math.npz")
    for (a, b), ref in zip(f["linspace_ab"], f["linspace_out"]):
        assert np.array_equal(O.linspace_torch(np.float32(a), np.float32(b), 50), ref)
    for x, s3, se3 in zip(f["sim3_in"], f["sim3_out"], f["se3_out"]):
        assert np.abs(O.exp_sim3(x) - s3).max() <= 2e-6
        assert np.abs(O.exp_se3(x[:6]) - se3).max() <= 2e-6
    rr, loss, w = O.get_robust_res(f["huber_res"].copy(), float(f["huber_b"]))
    assert np.abs(rr - f["huber_rr"]).max() <= 1e-7
    assert abs(loss - float(f["huber_loss"])) <= 1e-6 * float(f["huber_loss"])
    for T, ref in zip(f["rot_t_obj_cam"], f["rot_out"]):
        j, r = O.compute_rotation_loss_sim3(T)
        assert abs(float(r) - ref[7]) <= 1e-6
        assert np.abs(j - ref[:7]).max() <= 1e-5


@pytest.mark.slow
@pytest.mark.parametrize("name,optim", [("redwood0", S.REDWOOD_OPTIM), ("redwood1", S.REDWOOD_OPTIM)])
def test_teacher_forced_iterations(oracle_dec, name, optim):
    """F4: from every recorded reference state, one oracle GN step matches the reference's."""
    f = golden(f"f4_traj_{name}.npz")
    P = O.OptimParams.from_cfg(optim)
    n_fg = f["obj_depth"].shape[0]
    dobs = np.concatenate([f["obj_depth"], np.zeros(f["obj_rays"].shape[0] - n_fg)]).astype(np.float32)
    jo = optim["joint_optim"]
    for e in range(int(f["n_iters_run"])):
        tr, _, _ = O.gn_step(oracle_dec, P, f["it_t_obj_cam"][e], f["it_z"][e], f["obj_pts"],
                             f["obj_rays"], dobs, n_fg)
        # depth samples: same formula; endpoints differ by <= 1 ulp (numpy vs torch 4x4 LU)
        assert np.abs(O.linspace_torch(*_dminmax(f["it_t_obj_cam"][e]), 50)
                      - f["it_depths"][e]).max() <= 4e-7 * np.abs(f["it_depths"][e]).max()
        assert tr.n_valid == f["it_n_valid"][e]
        assert abs(tr.k - f["it_k"][e]) <= 2
        loss_ref = jo["k1"] * f["it_render_loss"][e] + jo["k2"] * f["it_sdf_loss"][e]
        assert abs(tr.loss - loss_ref) <= 1e-5 * abs(loss_ref)
        assert rel(tr.H, f["it_H"][e]) <= 3e-3
        assert rel(tr.b, f["it_b"][e]) <= 1e-2
        assert rel(tr.dx, f["it_dx"][e]) <= 2e-2


def _dminmax(t_obj_cam):
    t_cam_obj = np.linalg.inv(t_obj_cam)
    s = np.float32(np.linalg.det(t_cam_obj[:3, :3])) ** np.float32(1 / 3)
    return t_cam_obj[2, 3] - s, t_cam_obj[2, 3] + s


def test_reference_spread_fixture_is_consistent():
    """The ensemble (other thread counts / 1-ulp pose perturbations) is recorded and
    brackets a non-trivial spread: the noise floor for trajectory parity."""
    for name in ("redwood0", "redwood1", "kitti0", "kitti5"):
        f = golden(f"f4_traj_{name}.npz")
        assert f["ens_loss"].shape[0] >= 4
        assert np.isfinite(f["ens_loss"]).all()


def test_config4_ensemble_fixture_is_consistent():
    """F12 (tests/golden/make_ens4096.py): the F4 4096-point object at the full 10 iterations, the
    members' starts are the shared ulp-perturbation generator's, every member and the unperturbed
    run are good, and the unperturbed loss sits inside the members' spread."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_ensemble import member_poses

    f = golden("f12_ens_kitti4096.npz")
    f4 = golden("f4_traj_kitti4096.npz")
    assert np.array_equal(f["obj_pts"], f4["obj_pts"]) and int(f["num_iterations"]) == 10
    assert f["obj_pts"].shape == (4096, 3) and f["obj_rays"].shape == (4296, 3)
    assert np.array_equal(f["ens64_t_init"], member_poses(f["obj_t_cam_obj"], 64))
    assert bool(f["is_good"]) and bool(np.all(f["ens64_is_good"]))
    lo, hi = f["ens64_loss"].min(), f["ens64_loss"].max()
    assert lo <= float(f["loss"]) <= hi and hi - lo < 0.05 * float(f["loss"])


@pytest.mark.parametrize("name", ["kitti0", "kitti5"])
def test_exact_arithmetic_ensemble_fixtures_are_consistent(name):
    """F13 / F16 / F18 / F19 (tests/golden/make_ens256.py, tools/oracle_ens256.py): the reference's
    256-member 1-thread ensemble, the fp32 oracle's, the reference's 8-thread 64-member one and the
    fp64 oracle's (exact arithmetic) start from the same ulp-perturbed poses (the shared
    generator's); at iteration 0 — one state for every member — the three fp32 clouds and exact
    arithmetic agree to fp32 rounding (loss within 2e-4 relative, K within 2 render points), and
    every member of every cloud is good over its 10 iterations."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_ensemble import member_poses

    f4 = golden(f"f4_traj_{name}.npz")
    ref, orc, t8, ex = (golden(g) for g in (f"f13_ens256_{name}.npz", f"f16_oracle_ens256_{name}.npz",
                                            f"f18_ens64_t8_{name}.npz", f"f19_oracle64_ens64_{name}.npz"))
    assert np.array_equal(ref["t_init"], member_poses(f4["obj_t_cam_obj"], 256))
    assert np.array_equal(t8["t_init"], ref["t_init"][:64]) and int(t8["threads"]) == 8
    for g in (ref, orc, t8, ex):
        assert bool(np.all(g["is_good"])) and (g["it_k"] >= 0).all() and g["it_k"].shape[1] == 10
    lx = (ex["it_render_loss"] + 100.0 * ex["it_sdf_loss"])[:, 0]
    for g in (ref, orc, t8):
        lg = (g["it_render_loss"] + 100.0 * g["it_sdf_loss"])[:64, 0]
        assert np.abs(lg / lx - 1.0).max() <= 2e-4
        assert np.abs(g["it_k"][:64, 0].astype(np.int64) - ex["it_k"][:, 0]).max() <= 2


def test_failure_semantics():
    """F6: the reference returns is_good=False, loss = previous (0. at iteration 0)."""
    f = golden("f6_fail.npz")
    assert not bool(f["few_is_good"]) and float(f["few_loss"]) == 0.0
    assert int(f["few_iters"]) == 1


def test_failure_few_points_oracle(oracle_dec):
    f = golden("f6_fail.npz")
    P = O.OptimParams.from_cfg(S.REDWOOD_OPTIM)
    r = O.reconstruct_object(oracle_dec, P, f["few_t_cam_obj"], f["obj_pts"], f["obj_rays"],
                             f["obj_depth"])
    assert r.is_good == bool(f["few_is_good"]) and r.loss == float(f["few_loss"])


def test_zhjd_and_pose_only(oracle_dec):
    """F7: compute_sdf_loss_objectpoint_zhjd and estimate_pose_cam_obj."""
    f = golden("f7_secondary.npz")
    v = O.compute_sdf_loss_objectpoint(oracle_dec, f["zhjd_pts"], f["code"])
    assert abs(float(v) - float(f["zhjd_out"])) <= 2e-6
    P = O.OptimParams.from_cfg(S.KITTI_OPTIM)
    T = O.estimate_pose_cam_obj(oracle_dec, P, f["t_se3"], float(f["scale"]), f["pts"], f["code"])
    assert np.abs(T - f["pose_only_out"]).max() <= 1e-4 * np.abs(f["pose_only_out"]).max()


def _f8_paths():
    import glob
    import os

    from conftest import GOLDEN

    return sorted(glob.glob(os.path.join(GOLDEN, "f8_margin_*.npz")))


@pytest.mark.parametrize("path", _f8_paths(), ids=lambda p: p.rsplit("/", 1)[-1][10:-4])
def test_oracle_final_state_on_margin_fixtures(oracle_dec, path):
    """The oracle (numpy fp32) meets the north-star output contract against the reference
    on the margin-screened trajectories (F8, tests/golden/make_margin.py): exact K every
    iteration, final pose / code <= 1e-3, loss <= 1e-4 relative (optimizer.py:202-205)."""
    from test_gpu_contract import CODE_TOL, LOSS_TOL, POSE_TOL, contract_errors, optim_of

    f = np.load(path, allow_pickle=False)
    optim, _ = optim_of(f)
    P = O.OptimParams.from_cfg(optim)
    r = O.reconstruct_object(oracle_dec, P, f["obj_t_cam_obj"], f["obj_pts"], f["obj_rays"],
                             f["obj_depth"])
    assert r.is_good
    n_it = int(f["n_iters_run"])
    assert [tr.k for tr in r.trace] == f["it_k"][:n_it].tolist()
    e_rot, e_t, e_z, e_l = contract_errors(r.t_cam_obj, r.code, r.loss, f)
    assert e_rot <= POSE_TOL and e_t <= POSE_TOL and e_z <= CODE_TOL and e_l <= LOSS_TOL, \
        (e_rot, e_t, e_z, e_l)


def test_kitti_margin_fixtures_run_the_rotation_prior():
    """The strict contract covers KITTI parameters (configs/config_kitti.json: upright prior
    k4 = 1e7) with the prior ACTIVE: at every iteration of every KITTI F8 fixture the
    reference's res_rot = 1 - (R_co e_y).(0,-1,0) (loss.py:169-192) is far above its 1e-7
    switch, and the fp32 switch decision keeps a recorded margin of >= 4 ulps."""
    from test_gpu_contract import optim_of

    paths = [p for p in _f8_paths() if str(np.load(p)["data_type"]) == "KITTI"]
    assert len(paths) >= 3
    for p in paths:
        f = np.load(p, allow_pickle=False)
        optim, _ = optim_of(f)
        assert optim["joint_optim"]["k4"] == 1e7
        n_it = int(f["n_iters_run"])
        assert n_it >= 2 and f["is_good"]
        for e in range(n_it):
            tco = np.linalg.inv(f["it_t_obj_cam"][e].astype(np.float64))
            r = tco[:3, :3] / np.cbrt(np.linalg.det(tco[:3, :3]))
            assert 1.0 + r[1, 1] > 1e-6, (p, e)
        assert (f["margin_rot_ulps"][:n_it] >= 4.0).all()


def _edge_case_inputs(f, c):
    """Golden F10 (tests/golden/make_edge.py): case ``c``'s (pts, rays, depth)."""
    n, nr, nf = int(f[c + "_n_pts"]), int(f[c + "_n_rays"]), int(f[c + "_n_fg"])
    n_fg_all = f["obj_depth"].shape[0]
    rays = f["obj_rays"][n_fg_all:] if c == "no_fg_rays" else f["obj_rays"][:nr]
    assert rays.shape[0] == nr
    return f["obj_pts"][:n], rays, f["obj_depth"][:nf]


def test_oracle_edge_cases_f10(oracle_dec):
    """Empty and ragged inputs (F10): no surface points / no rays fail like the reference
    (is_good False, loss 0. — optimizer.py:132-145), one point, background-only and
    foreground-only rays give the reference's trajectory (K each iteration, final loss);
    pose-only GN and the zhjd query on no points give NaN (optimizer.py:62-87, 207-213)."""
    f = golden("f10_edge.npz")
    P = O.OptimParams.from_cfg(dict(S.REDWOOD_OPTIM, joint_optim=dict(S.REDWOOD_OPTIM["joint_optim"],
                                                                        num_iterations=int(f["num_iterations"]))))
    for c in f["cases"]:
        c = str(c)
        pts, rays, depth = _edge_case_inputs(f, c)
        r = O.reconstruct_object(oracle_dec, P, f["obj_t_cam_obj"], pts, rays, depth)
        assert r.is_good == bool(f[c + "_is_good"]), c
        if not r.is_good:
            assert r.loss == 0.0 == float(f[c + "_loss"]) and r.t_cam_obj is None, c
            continue
        assert [t.k for t in r.trace] == f[c + "_it_k"].tolist(), c
        assert abs(r.loss - float(f[c + "_loss"])) <= 1e-4 * abs(float(f[c + "_loss"])), c
    Pk = O.OptimParams.from_cfg(S.KITTI_OPTIM)
    z = np.zeros(64, np.float32)
    T = O.estimate_pose_cam_obj(oracle_dec, Pk, f["pose_t_se3"], float(f["pose_scale"]), f["obj_pts"][:0], z)
    assert np.isnan(T).all() and np.isnan(f["pose_empty_out"]).all()
    assert np.isnan(O.compute_sdf_loss_objectpoint(oracle_dec, f["obj_pts"][:0], z)) and np.isnan(f["zhjd_empty_out"])


SPECS32 = dict(S.DEFAULT_SPECS, CodeLength=32)
KITTI32 = dict(S.KITTI_OPTIM, code_len=32, joint_optim=dict(S.KITTI_OPTIM["joint_optim"], num_iterations=3))


def test_oracle_code32_decoder_and_steps():
    """Golden F15 (tests/golden/make_code32.py: the REFERENCE with a CodeLength-32 decoder,
    /root/reference/src/LocalMapping_util.cc:416-422): the regenerated 32-D decoder folds to the
    reference's weights bit for bit, the oracle's sdf / Jacobian (35 columns) match its
    get_batch_sdf_jacobian, and one oracle GN step from each recorded reference state matches
    its 39-parameter H / b / dx and losses."""
    import hashlib

    from deep_sdf.workspace import fold_state

    f = golden("f15_code32.npz")
    layers = fold_state(S.make_decoder(1234, SPECS32), SPECS32)
    h = hashlib.sha256()
    for W, b in layers:
        h.update(W.tobytes())
        h.update(b.tobytes())
    assert h.hexdigest() == str(f["folded_sha256"])
    assert [W.shape for W, _ in layers][0] == (512, 35) and layers[3][0].shape == (477, 512)
    dec = O.Decoder(layers, 32, (4,))
    y, j = dec.forward_jac(np.concatenate([np.broadcast_to(f["z"], (256, 32)), f["x"]], 1))
    assert np.abs(y - f["sdf"]).max() <= 2e-6
    assert_jac_close(j, f["jac"], tol=2e-5)
    P = O.OptimParams.from_cfg(KITTI32)
    n_fg = f["obj_depth"].shape[0]
    dobs = np.concatenate([f["obj_depth"], np.zeros(f["obj_rays"].shape[0] - n_fg)]).astype(np.float32)
    jo = KITTI32["joint_optim"]
    assert f["it_H"].shape[1:] == (39, 39)
    for e in range(int(f["n_iters_run"])):
        tr, _, _ = O.gn_step(dec, P, f["it_t_obj_cam"][e], f["it_z"][e], f["obj_pts"], f["obj_rays"], dobs, n_fg)
        assert abs(tr.k - f["it_k"][e]) <= 2
        loss_ref = jo["k1"] * f["it_render_loss"][e] + jo["k2"] * f["it_sdf_loss"][e]
        assert abs(tr.loss - loss_ref) <= 1e-5 * abs(loss_ref)
        assert tr.H.shape == (39, 39)
        assert rel(tr.H, f["it_H"][e]) <= 3e-3
        assert rel(tr.b, f["it_b"][e]) <= 1e-2


def _variant_specs(v):
    import copy

    specs = copy.deepcopy(S.DEFAULT_SPECS)
    ns = specs["NetworkSpecs"]
    if v == "tanh":
        ns["use_tanh"] = True
    elif v == "xyz":
        ns["xyz_in_all"] = True
    elif v == "plain":
        ns["weight_norm"] = False
        ns["norm_layers"] = []
    else:                                    # "ln": LayerNorm after lin0..lin7
        ns["weight_norm"] = False
    return specs


@pytest.mark.parametrize("v", ["tanh", "xyz", "plain", "ln"])
def test_oracle_decoder_variants(v):
    """Golden F17 (tests/golden/make_variants.py: the REFERENCE's module with use_tanh,
    xyz_in_all, plain Linear or LayerNorm layers, deep_sdf_decoder.py:41-63, 89-102): the regenerated
    decoder folds to the reference's weights bit for bit, the oracle's sdf / Jacobian match
    get_batch_sdf_jacobian, and (all but plain) one oracle GN step from each recorded
    reference state matches its K, loss, H, b."""
    import hashlib

    from deep_sdf.workspace import check_topology, fold_state, norm_state

    f = golden("f17_variants.npz")
    specs = _variant_specs(v)
    layers = fold_state(S.make_decoder(1234, specs), specs)
    check_topology(specs, layers)
    h = hashlib.sha256()
    for W, b in layers:
        h.update(W.tobytes())
        h.update(b.tobytes())
    for n in norm_state(S.make_decoder(1234, specs), specs):
        if n is not None:
            h.update(n[0].tobytes())
            h.update(n[1].tobytes())
    assert h.hexdigest() == str(f[v + "_folded_sha256"])
    dec = O.Decoder.from_state(S.make_decoder(1234, specs), specs)
    y, j = dec.forward_jac(np.concatenate([np.broadcast_to(f[v + "_z"], (256, 64)), f[v + "_x"]], 1))
    assert np.abs(y - f[v + "_sdf"]).max() <= 2e-6
    assert_jac_close(j, f[v + "_jac"], tol=2e-5)
    assert np.abs(O.decode_sdf(dec, f[v + "_z"], f[v + "_x"]) - f[v + "_sdf_nograd"]).max() <= 2e-6
    if v == "plain":
        return
    P = O.OptimParams.from_cfg(S.KITTI_OPTIM)
    n_fg = f[v + "_obj_depth"].shape[0]
    dobs = np.concatenate([f[v + "_obj_depth"], np.zeros(f[v + "_obj_rays"].shape[0] - n_fg)]).astype(np.float32)
    jo = S.KITTI_OPTIM["joint_optim"]
    for e in range(int(f[v + "_n_iters_run"])):
        tr, _, _ = O.gn_step(dec, P, f[v + "_it_t_obj_cam"][e], f[v + "_it_z"][e], f[v + "_obj_pts"],
                             f[v + "_obj_rays"], dobs, n_fg)
        dk = abs(tr.k - int(f[v + "_it_k"][e]))
        assert dk <= 2
        loss_ref = jo["k1"] * f[v + "_it_render_loss"][e] + jo["k2"] * f[v + "_it_sdf_loss"][e]
        # (+ the most one flipped render point moves the render term, as in test_gpu_parity)
        assert abs(tr.loss - loss_ref) <= 1e-5 * abs(loss_ref) + dk * jo["k1"] * 0.09 / f[v + "_it_k"][e]
        assert rel(tr.H, f[v + "_it_H"][e]) <= (3e-3 if dk == 0 else 1e-2)
        assert rel(tr.b, f[v + "_it_b"][e]) <= (1e-2 if dk == 0 else 3e-2)


def test_f8_conditioning_record_reproduces():
    """tests/golden/f8_conditioning.json (tools/f8_conditioning.py), which the strict GPU contract
    test reads to tell a well-conditioned margin fixture from one whose GN step amplifies an
    fp32-sized state error out of the contract: the ill-conditioned entry (redwood_s5359,
    iteration 2: the fp32 oracle's own 2e-6 state error -> 1.9e-2 in the next state) and one
    well-conditioned entry recomputed here with the fp64 oracle, same seed."""
    import json
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
    import f8_conditioning as FC

    rec = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "f8_conditioning.json")))
    d64, d32 = FC.decoders()
    for name in ("redwood_s5359", "redwood3it_s5006"):
        c = FC.conditioning(os.path.join(os.path.dirname(__file__), "golden", f"f8_margin_{name}.npz"), d64, d32)
        r = rec["fixtures"][name]
        assert c["well_conditioned"] == r["well_conditioned"], name
        np.testing.assert_allclose(c["worst_next_state_deviation"], r["worst_next_state_deviation"], rtol=1e-6)
    assert not rec["fixtures"]["redwood_s5359"]["well_conditioned"]
    assert rec["fixtures"]["redwood_s5359"]["worst_next_state_deviation"][2] > 1e-2
    assert sum(e["well_conditioned"] for e in rec["fixtures"].values()) >= 9
