"""HIP path (libdsr.so via ctypes) vs the reference's golden vectors and the oracle.

Tolerances:
* decoder SDF / Jacobian vs golden F1: fp32, |err| <= 2e-5 abs (sdf in (-1,1)),
  <= 1e-4 x max|jac| for the Jacobian (autograd vs analytic backward, fp32 sums);
* one teacher-forced GN iteration vs golden F4 (same state in): N_valid and K within
  2 (samples within fp32 rounding of |x| = 1 or |sdf| = th flip between any two fp32
  implementations; the loss bound grows by the most one flipped render point can move
  it), loss rel <= 1e-5 at identical K, H and b (all but b[3:6]) <= 5e-4 at identical K
  (<= 2e-3 / 5e-3 with a flipped render point), b[3:6] and dx <= 5e-2 max-normalised and
  the step <= 1e-2 in the H-norm (b[3:6] carries k4 * J_rot * r_rot with k4 = 1e7 and
  r_rot an fp32 cancellation quantised in 6e-8 steps, in the reference itself);
* full trajectories: mask flips (|sdf|=th, de_do=1e-2, |x|=1) and ReLU kinks at the
  Jacobian points amplify fp32 rounding chaotically — the reference itself moves by
  up to 4e-1 in its final code under a 1-ulp pose perturbation (F4 ensembles).  The
  trajectory test therefore checks every GPU step against the oracle's step FROM THE
  GPU'S OWN STATE (shadowing); the final state is held to the reference in
  tests/test_gpu_contract.py (strictly on margin-screened inputs, by the reference's
  own reproducibility envelope on these).
"""
from __future__ import annotations

import numpy as np
import pytest

import synthetic as S
from conftest import assert_jac_close, golden, make_cfg

pytestmark = pytest.mark.gpu


def _opt(dec, optim, data_type="KITTI"):
    from reconstruct.optimizer import Optimizer

    return Optimizer(dec, make_cfg(optim, data_type))


def rel(a, b):
    return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


def step_err(dx, dx_ref, H):
    """GN step error in the H-norm, sqrt(d'Hd / dx'H dx): insensitive to the badly
    determined directions (e.g. yaw of a near-rotationally-symmetric shape) where the
    quadratic model is flat and tiny b differences move dx a lot at no cost."""
    d = np.asarray(dx, np.float64) - dx_ref
    H = np.asarray(H, np.float64)
    return float(np.sqrt(max(d @ H @ d, 0.0) / max(dx_ref @ H @ dx_ref, 1e-300)))


def test_library_is_native(gpu_decoder):
    from reconstruct import _libdsr as L

    lib = L.load_library()
    n = L.C.c_int()
    assert lib.dsr_device_count(L.C.byref(n)) == 0 and n.value >= 1
    assert gpu_decoder.handle


@pytest.mark.parametrize("n", [1, 63, 256, 1000])
def test_decoder_fwd_jac_vs_golden(gpu_decoder, n):
    from reconstruct.optimizer import sdf_eval

    g = golden("f1_decoder_full.npz")
    x = np.resize(g["x"], (n, 3))
    y_ref = np.resize(g["sdf"], n)
    j_ref = np.resize(g["jac"], (n, 67))
    y, j = sdf_eval(gpu_decoder, g["z"], x, with_jac=True)
    assert np.abs(y - y_ref).max() <= 2e-5
    assert_jac_close(j, j_ref, tol=1e-4)
    y2 = sdf_eval(gpu_decoder, g["z"], x)
    assert np.abs(y2 - np.resize(g["sdf_nograd"], n)).max() <= 2e-5
    # forward-only and fwd+jac kernels compute the same forward
    assert np.abs(y2 - y).max() <= 1e-6


def test_decoder_vs_oracle_random(gpu_decoder, oracle_dec):
    from reconstruct.optimizer import sdf_eval

    rng = np.random.default_rng(5)
    z = (0.2 * rng.standard_normal(64)).astype(np.float32)
    x = rng.uniform(-1, 1, (3000, 3)).astype(np.float32)
    y, j = sdf_eval(gpu_decoder, z, x, with_jac=True)
    inp = np.concatenate([np.broadcast_to(z, (3000, 64)), x], 1)
    y64, j64 = type(oracle_dec)(oracle_dec.layers, dtype=np.float64).forward_jac(inp.astype(np.float64))
    assert np.abs(y - y64).max() <= 2e-5
    assert_jac_close(j, j64, tol=1e-4)


@pytest.mark.parametrize("name,optim,dtype", [("redwood0", S.REDWOOD_OPTIM, "Redwood"),
                                              ("redwood1", S.REDWOOD_OPTIM, "Redwood"),
                                              ("kitti0", S.KITTI_OPTIM, "KITTI"),
                                              ("kitti5", S.KITTI_OPTIM, "KITTI"),
                                              ("kitti4096", S.KITTI_OPTIM, "KITTI")])
def test_teacher_forced_iterations_vs_golden(gpu_decoder, name, optim, dtype):
    """Every recorded reference state -> one GPU GN step -> H, b, dx, loss, K."""
    f = golden(f"f4_traj_{name}.npz")
    one = dict(optim, joint_optim=dict(optim["joint_optim"], num_iterations=1))
    opt = _opt(gpu_decoder, one, dtype)
    n_it = int(f["n_iters_run"])
    objs = [(f["it_t_obj_cam"][e], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][e])
            for e in range(n_it)]
    res, tr = opt.reconstruct_objects(objs, trace=True, pose_is_obj_cam=True)
    jo = optim["joint_optim"]
    for e in range(n_it):
        t = tr[e]
        assert res[e]["is_good"], (e, res[e])
        assert abs(int(t["n_valid"][0]) - int(f["it_n_valid"][e])) <= 2
        assert abs(int(t["k"][0]) - int(f["it_k"][e])) <= 2
        loss_ref = jo["k1"] * f["it_render_loss"][e] + jo["k2"] * f["it_sdf_loss"][e]
        # identical render set -> 1e-5; each flipped render point moves the mean Huber
        # loss by at most (2 b1 0.3 - b1^2)/K <= 0.09/K (clamp +-0.30, loss.py:147-148)
        dk = abs(int(t["k"][0]) - int(f["it_k"][e]))
        tol = 1e-5 * abs(loss_ref) + dk * jo["k1"] * 0.09 / f["it_k"][e]
        assert abs(t["loss"][0] - loss_ref) <= tol, (e, dk)
        if dk == 0:
            assert abs(t["render_loss"][0] - f["it_render_loss"][e]) <= 1e-5 * f["it_render_loss"][e]
            # the sdf residuals are surface-point SDFs ~1e-2 while any fp32 decoder is off
            # by ~1e-7 absolute (numpy fp32 vs fp64: rms 7.6e-8, tools/diag_precision.py),
            # so mean(r^2) carries ~2e-5 relative noise in every fp32 implementation
            assert abs(t["sdf_loss"][0] - f["it_sdf_loss"][e]) <= 5e-5 * f["it_sdf_loss"][e]
        eh = rel(t["H"][0], f["it_H"][e])
        # b[3:6] carries k4 * J_rot * r_rot with k4 = 1e7 and r_rot = 1 - cos(tilt), an fp32
        # cancellation in the reference itself (quantised in 6e-8 steps): those three entries
        # are held loosely, the other 68 like H; dx in the H-norm (the step GN takes)
        rest = np.r_[0:3, 6:71]
        eb = rel(np.asarray(t["b"][0])[rest], np.asarray(f["it_b"][e])[rest])
        eb_rot = rel(t["b"][0], f["it_b"][e])
        es = step_err(t["dx"][0], f["it_dx"][e], f["it_H"][e])
        edx = rel(t["dx"][0], f["it_dx"][e])
        print(f"{name} it {e}: dK {dk} H {eh:.2e} b {eb:.2e} b(all) {eb_rot:.2e} dx(H-norm) {es:.2e} dx {edx:.2e}")
        # measured (r2, every F4 state): identical K -> H <= 1.2e-4, b <= 1.4e-4; one flipped
        # render point -> H <= 2.4e-4, b <= 1.5e-3; dx <= 9.9e-3 in the H-norm.  b[3:6] and dx
        # max-normalised are held against the fp64 truth below
        # (test_teacher_forced_steps_no_less_accurate_than_the_reference)
        assert eh <= (5e-4 if dk == 0 else 2e-3), (e, eh)
        assert eb <= (5e-4 if dk == 0 else 5e-3), (e, eb)
        assert es <= 1e-2, e


@pytest.mark.parametrize("name,optim,dtype", [("redwood0", S.REDWOOD_OPTIM, "Redwood"),
                                              ("redwood1", S.REDWOOD_OPTIM, "Redwood"),
                                              ("kitti0", S.KITTI_OPTIM, "KITTI"),
                                              ("kitti5", S.KITTI_OPTIM, "KITTI"),
                                              ("kitti4096", S.KITTI_OPTIM, "KITTI")])
def test_teacher_forced_steps_no_less_accurate_than_the_reference(gpu_decoder, name, optim, dtype):
    """from every recorded reference state, the GPU's b — in particular
    b[3:6], where the rotation prior puts k4 = 1e7 times an fp32 cancellation (r_rot = 1 - cos
    of the tilt, /root/reference/reconstruct/loss.py:169-192, optimizer.py:176-181) — and its
    step dx are measured against the fp64 truth of the same step (golden F14: the oracle in
    float64 from that state, tests/golden/make_fp64_truth.py), and so is the reference's own fp32
    b / dx (F4 it_b / it_dx), at every iteration whose render set K agrees in all three.

    Criterion (set from the r4d/r4e measurements, tools/acc_probe.py): per
    iteration both fp32 implementations show isolated 10-100x error spikes — a Jacobian point
    whose ReLU pre-activation or Huber residual sits within rounding of its kink takes the
    other branch — and they land on either side (redwood0: GPU 4.3e-4 vs reference 6.4e-6 on
    b[3:6] at iteration 3, reference 1.8e-3 vs GPU 3.2e-5 at iteration 4), so no per-iteration
    ratio can hold.  Held instead: over the trajectory, the RMS error of b[3:6], dx and dx in
    the H-norm within 1.25x the reference's; b's other entries within 2x (the split-fp16
    decode carries 22-bit operands: 1.2-1.8x the reference's RMS there, where the fp32-MFMA
    kernels give 1.0-1.2x — it does not reach dx); and no single iteration beyond 2x the
    reference's largest error over the trajectory."""
    f = golden(f"f4_traj_{name}.npz")
    t64 = golden(f"f14_fp64_{name}.npz")
    one = dict(optim, joint_optim=dict(optim["joint_optim"], num_iterations=1))
    opt = _opt(gpu_decoder, one, dtype)
    n_it = int(f["n_iters_run"])
    objs = [(f["it_t_obj_cam"][e], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][e])
            for e in range(n_it)]
    res, tr = opt.reconstruct_objects(objs, trace=True, pose_is_obj_cam=True)
    eps = 2.0 ** -23
    acc = {k: [] for k in ("b_rot", "b_rest", "dx", "dx_H")}
    used = 0
    for e in range(n_it):
        kg, kr, k64 = int(tr[e]["k"][0]), int(f["it_k"][e]), int(t64["k"][e])
        if not (kg == kr == k64):
            print(f"{name} it {e}: K gpu {kg} ref {kr} fp64 {k64} (skipped: different render sets)")
            continue
        used += 1
        b64, dx64, H64 = (np.asarray(t64[k][e], np.float64) for k in ("b", "dx", "H"))
        rows = []
        for key, sl in (("b_rot", np.s_[3:6]), ("b_rest", np.r_[0:3, 6:71])):
            sc = np.abs(b64[sl]).max()
            eg = np.abs(np.asarray(tr[e]["b"][0], np.float64)[sl] - b64[sl]).max() / sc
            er = np.abs(np.asarray(f["it_b"][e], np.float64)[sl] - b64[sl]).max() / sc
            acc[key].append((eg, er))
            rows.append(f"{key} gpu {eg:.2e} ref {er:.2e}")
        sc = np.abs(dx64).max()
        eg = np.abs(np.asarray(tr[e]["dx"][0], np.float64) - dx64).max() / sc
        er = np.abs(np.asarray(f["it_dx"][e], np.float64) - dx64).max() / sc
        acc["dx"].append((eg, er))
        hg = step_err(tr[e]["dx"][0], dx64, H64)
        hr = step_err(f["it_dx"][e], dx64, H64)
        acc["dx_H"].append((hg, hr))
        print(f"{name} it {e}: " + "  ".join(rows) + f"  dx gpu {eg:.2e} ref {er:.2e}  dx(H) gpu {hg:.2e} ref {hr:.2e}")
    assert used >= max(1, n_it // 2), (used, n_it)
    for key, v in acc.items():
        a = np.array(v)
        rms_g, rms_r = np.sqrt((a[:, 0] ** 2).mean()), np.sqrt((a[:, 1] ** 2).mean())
        print(f"{name} {key}: RMS error vs fp64 gpu {rms_g:.2e} ref {rms_r:.2e}; worst gpu {a[:, 0].max():.2e} "
              f"ref {a[:, 1].max():.2e}")
        assert a[:, 0].max() <= 2.0 * a[:, 1].max() + 4 * eps, (key, a[:, 0].max(), a[:, 1].max())
        assert rms_g <= (2.0 if key == "b_rest" else 1.25) * rms_r + 4 * eps, (key, rms_g, rms_r)


@pytest.mark.parametrize("name,optim,dtype", [("redwood0", S.REDWOOD_OPTIM, "Redwood"),
                                              ("redwood1", S.REDWOOD_OPTIM, "Redwood"),
                                              ("kitti0", S.KITTI_OPTIM, "KITTI"),
                                              ("kitti5", S.KITTI_OPTIM, "KITTI")])
def test_trajectory_shadowing_and_final(gpu_decoder, oracle_dec, name, optim, dtype):
    """Full GPU trajectory; every GPU step re-checked against the oracle from the GPU state."""
    from oracle import dsr_oracle as O

    f = golden(f"f4_traj_{name}.npz")
    opt = _opt(gpu_decoder, optim, dtype)
    (r,), (t,) = opt.reconstruct_objects(
        [(f["obj_t_cam_obj"], f["obj_pts"], f["obj_rays"], f["obj_depth"], None)], trace=True)
    assert r["is_good"]
    # (final state vs the reference: test_gpu_contract.py)
    # shadowing: the GPU's step e, re-taken from the state the GPU itself reached, vs
    # the oracle's step from that same state
    P = O.OptimParams.from_cfg(optim)
    one = dict(optim, joint_optim=dict(optim["joint_optim"], num_iterations=1))
    opt1 = _opt(gpu_decoder, one, dtype)
    n_fg = f["obj_depth"].shape[0]
    dobs = np.concatenate([f["obj_depth"], np.zeros(f["obj_rays"].shape[0] - n_fg)]).astype(np.float32)
    n_it = int(f["n_iters_run"])
    for e in sorted({0, n_it // 2, n_it - 1}):
        state_T, z = t["t_obj_cam"][e], t["z"][e]
        (rg,), (tg,) = opt1.reconstruct_objects(
            [(state_T, f["obj_pts"], f["obj_rays"], f["obj_depth"], z)], trace=True,
            pose_is_obj_cam=True)
        assert tg["loss"][0] == t["loss"][e]          # re-running a state is deterministic
        tro, _, _ = O.gn_step(oracle_dec, P, state_T, z, f["obj_pts"], f["obj_rays"], dobs, n_fg)
        assert abs(tg["k"][0] - tro.k) <= 2
        assert abs(int(tg["n_valid"][0]) - tro.n_valid) <= 2
        # terms separately, as in the teacher-forced test: the sdf term carries only fp32
        # decoder noise; the render term additionally moves by <= 0.09/K per render point
        # that flips across |sdf| = th or de_do = 1e-2 (clamp +-0.30, loss.py:147-148) — a
        # flip can swap points without changing K, so allow up to 2 of them
        jo = optim["joint_optim"]
        assert abs(tg["sdf_loss"][0] - tro.sdf_loss) <= 5e-5 * abs(tro.sdf_loss)
        flips = max(abs(int(tg["k"][0]) - tro.k), 2)
        assert abs(tg["render_loss"][0] - tro.render_loss) <= (1e-5 * abs(tro.render_loss)
                                                              + flips * 0.09 / tro.k), (e, tg["k"][0], tro.k)
        assert abs(tg["loss"][0] - tro.loss) <= (1e-4 * abs(tro.loss)
                                                 + jo["k1"] * flips * 0.09 / tro.k)
        assert rel(tg["H"][0], tro.H) <= 5e-3
        assert step_err(tg["dx"][0], tro.dx, tro.H) <= 2e-2
    assert np.isfinite(t["loss"]).all()


@pytest.mark.parametrize("streams", ["1", "2", "3", "4"])
def test_batch_equals_single(gpu_decoder, streams, monkeypatch):
    """Objects in a batch are independent: batched results == one-by-one, bitwise, however
    the batch is split into object groups on concurrent streams (DSR_STREAMS).  The schedule is
    pinned here so that each object-group count runs the same windows; that the default
    schedules themselves change no bit is test_default_schedules_give_bitwise_equal_results."""
    monkeypatch.setenv("DSR_STREAMS", streams)
    monkeypatch.setenv("DSR_TEST_HOOKS", "1")   # kernel switches are test hooks
    monkeypatch.setenv("DSR_RENDER_PASSES", "16,24")
    opt = _opt(gpu_decoder, dict(S.REDWOOD_OPTIM, joint_optim=dict(S.REDWOOD_OPTIM["joint_optim"],
                                                                    num_iterations=3)), "Redwood")
    objs = []
    for i in range(5):
        o = S.make_object(300 + i, n_pts=200 + 97 * i, n_bg=50 + 10 * i, scale=1.0, tz=3.0,
                          upright=False)
        objs.append((o.t_cam_obj, o.pts, o.rays, o.depth, None))
    batch, tr = opt.reconstruct_objects(objs, trace=True)
    for i, ob in enumerate(objs):
        single, tr1 = opt.reconstruct_objects([ob], trace=True)
        single = single[0]
        assert batch[i]["is_good"] == single["is_good"]
        if single["is_good"]:
            assert np.array_equal(batch[i]["t_cam_obj"], single["t_cam_obj"])
            assert np.array_equal(batch[i]["code"], single["code"])
            assert batch[i]["loss"] == single["loss"]
        for key in ("H", "b", "loss", "n_valid", "k"):
            assert np.array_equal(tr[i][key], tr1[0][key]), (i, key)


def test_default_schedules_give_bitwise_equal_results(gpu_decoder, monkeypatch):
    """the default render-pass schedule depends on the batch's sample
    count, ray count and the device's CU count — so an object alone (one KITTI object: windows
    20), in an 8-object shard (16,24), in a 16-object frame (8,12,16,20,24,32) or decoded in
    ONE pass gets a different schedule.  None of this may change a bit of its result: the lite
    values are per sample, every sample in front of a ray's first certainly-full one is decoded
    under every schedule, and the exact pass re-decodes exactly those flagged in front of it
    (band, audit shell and the hashed audits: k_refine_scan stops there), so its tiles — and
    their split-fp16 scales — are the same list under every schedule."""
    monkeypatch.delenv("DSR_RENDER_PASSES", raising=False)
    monkeypatch.delenv("DSR_STREAMS", raising=False)
    opt = _opt(gpu_decoder, dict(S.KITTI_OPTIM, joint_optim=dict(S.KITTI_OPTIM["joint_optim"], num_iterations=3)),
               "KITTI")
    objs = [(o.t_cam_obj, o.pts, o.rays, o.depth, None) for o in (S.kitti_object(i) for i in range(16))]
    runs = {"batch16": opt.reconstruct_objects(objs, trace=True),
            "batch8": opt.reconstruct_objects(objs[:8], trace=True)}
    singles = [opt.reconstruct_objects([ob], trace=True) for ob in objs[:3]]
    monkeypatch.setenv("DSR_TEST_HOOKS", "1")   # kernel switches are test hooks
    monkeypatch.setenv("DSR_RENDER_PASSES", "0")
    runs["one_pass"] = opt.reconstruct_objects(objs[:8], trace=True)
    monkeypatch.delenv("DSR_RENDER_PASSES")
    # the object groups' slices packed back to back instead of line-aligned;
    # one group with the first pass's chunked ray scan (its default) and without it
    monkeypatch.setenv("DSR_GROUP_ALIGN", "0")
    runs["packed"] = opt.reconstruct_objects(objs[:8], trace=True)
    monkeypatch.delenv("DSR_GROUP_ALIGN")
    monkeypatch.setenv("DSR_STREAMS", "1")
    runs["one_group_scan"] = opt.reconstruct_objects(objs[:8], trace=True)
    monkeypatch.setenv("DSR_PRESCAN", "0")
    runs["one_group_no_scan"] = opt.reconstruct_objects(objs[:8], trace=True)
    ref_res, ref_tr = runs["batch8"]
    cases = [(k, runs[k], range(8)) for k in ("batch16", "one_pass", "packed", "one_group_scan", "one_group_no_scan")]
    cases += [(f"single{i}", singles[i], [i]) for i in range(len(singles))]
    # per-object work counts: the exact pass's sample list is the same under
    # every schedule, so each object's refined-sample count is too; the decoded-sample count
    # depends on the pass windows only (samples behind a ray's first certainly-full one), so
    # the schedules with batch8's windows — the packed groups, one group with and without the
    # chunked first-pass scan — must decode exactly batch8's samples, object by object
    same_windows = ("packed", "one_group_scan", "one_group_no_scan")
    for name, (res, tr), idx in cases:
        for j, i in enumerate(idx):
            a, b = res[j], ref_res[i]
            assert a["is_good"] == b["is_good"] and a["loss"] == b["loss"], (name, i)
            if a["is_good"]:
                assert np.array_equal(a["t_cam_obj"], b["t_cam_obj"]), (name, i)
                assert np.array_equal(a["code"], b["code"]), (name, i)
            for key in ("H", "b", "n_valid", "k", "n_refined") + (("n_decoded",) if name in same_windows else ()):
                assert np.array_equal(tr[j][key], ref_tr[i][key]), (name, i, key)
    assert ref_tr[0]["n_decoded"].min() > 0 and ref_tr[0]["n_refined"].min() > 0


def test_chunked_scan_with_four_groups_decodes_the_same_samples_every_run(gpu_decoder, monkeypatch):
    """VERDICT r5 item 1 / DESIGN.md §3.9: the chunked first-pass ray scan (k_sample_scan) with
    four object groups on their own streams — the setting whose decoded-sample counts varied in
    7-8 of 16 runs in round 5 — must decode, object by object and iteration by iteration, exactly
    the samples the scan-free sequence decodes, in every run.  The cause was wrong products of a
    packed-FP32 multiply in the scan loop's first trip (one quarter-wave, ~1 run in 10, only beside
    other groups' decoder kernels); the ray-sample kernels are built without packed FP32 now."""
    monkeypatch.setenv("DSR_TEST_HOOKS", "1")
    monkeypatch.setenv("DSR_STREAMS", "4")
    monkeypatch.delenv("DSR_RENDER_PASSES", raising=False)
    opt = _opt(gpu_decoder, S.KITTI_OPTIM, "KITTI")
    objs = [(o.t_cam_obj, o.pts, o.rays, o.depth, None) for o in (S.kitti_object(i) for i in range(8))]
    monkeypatch.setenv("DSR_PRESCAN", "0")
    ref_res, ref_tr = opt.reconstruct_objects(objs, trace=True)
    monkeypatch.setenv("DSR_PRESCAN", "1")
    for run in range(8):
        res, tr = opt.reconstruct_objects(objs, trace=True)
        for i in range(8):
            assert res[i]["loss"] == ref_res[i]["loss"], (run, i)
            for key in ("n_decoded", "n_refined", "n_valid", "k", "H", "b"):
                assert np.array_equal(tr[i][key], ref_tr[i][key]), (run, i, key)


def test_chunked_render_passes_match_the_per_object_pass_on_ragged_rays(gpu_decoder, monkeypatch):
    """The render passes over ray chunks (k_sample_scan / k_sample_count + k_sample_emit, one
    group) against the one-workgroup-per-object k_sample_pass (DSR_PRESCAN=0) on objects whose ray
    counts straddle the 128-ray chunks — none, one, a few, 127 / 128 / 129, a partial last chunk,
    a full KITTI object: bitwise equal results and per-iteration decoded / refined counts,
    N_valid, K, H, b.  The ray-less object fails in its first iteration with loss 0 (no in-ball
    samples: loss.py:86-88, optimizer.py:119, 144-145) — in k_iter_begin on the chunked path,
    which has no workgroup for it."""
    monkeypatch.setenv("DSR_TEST_HOOKS", "1")
    monkeypatch.setenv("DSR_STREAMS", "1")
    monkeypatch.delenv("DSR_RENDER_PASSES", raising=False)
    opt = _opt(gpu_decoder, dict(S.KITTI_OPTIM, joint_optim=dict(S.KITTI_OPTIM["joint_optim"], num_iterations=3)),
               "KITTI")
    objs = []
    for i, nr in enumerate((0, 1, 5, 127, 128, 129, 300, 2248)):
        o = S.kitti_object(20 + i)
        rays = np.ascontiguousarray(o.rays[:nr])
        objs.append((o.t_cam_obj, o.pts, rays, np.ascontiguousarray(o.depth[:min(nr, o.depth.shape[0])]), None))
    runs = {}
    for pre in ("1", "0"):
        monkeypatch.setenv("DSR_PRESCAN", pre)
        runs[pre] = opt.reconstruct_objects(objs, trace=True)
    (ra, ta), (rb, tb) = runs["1"], runs["0"]
    for i in range(len(objs)):
        a, b = ra[i], rb[i]
        assert a["is_good"] == b["is_good"] and a["loss"] == b["loss"], i
        if a["is_good"]:
            assert np.array_equal(a["t_cam_obj"], b["t_cam_obj"]) and np.array_equal(a["code"], b["code"]), i
        for key in ("H", "b", "n_valid", "k", "n_decoded", "n_refined"):
            assert np.array_equal(ta[i][key], tb[i][key]), (i, key)
    assert not ra[0]["is_good"] and ra[0]["loss"] == 0.0, ra[0]
    assert ra[7]["is_good"] and ta[7]["n_decoded"].min() > 0 and ta[7]["n_refined"].min() > 0


def test_failure_cases(gpu_decoder):
    f = golden("f6_fail.npz")
    opt = _opt(gpu_decoder, S.REDWOOD_OPTIM, "Redwood")
    r = opt.reconstruct_object(f["few_t_cam_obj"], f["obj_pts"], f["obj_rays"], f["obj_depth"])
    assert r["is_good"] == bool(f["few_is_good"])
    assert r["t_cam_obj"] is None and r["code"] is None
    assert r["loss"] == float(f["few_loss"])
    r = opt.reconstruct_object(f["obj_t_cam_obj"], f["obj_pts"], f["obj_rays"], f["obj_depth"],
                               f["bigcode"])
    assert r["is_good"] == bool(f["bigcode_is_good"])
    if not r["is_good"]:
        assert abs(r["loss"] - float(f["bigcode_loss"])) <= 1e-3 * max(1.0, abs(float(f["bigcode_loss"])))


def test_warm_start_code(gpu_decoder):
    f = golden("f6_fail.npz")
    opt = _opt(gpu_decoder, S.REDWOOD_OPTIM, "Redwood")
    r = opt.reconstruct_object(f["obj_t_cam_obj"], f["obj_pts"], f["obj_rays"], f["obj_depth"],
                               f["warm_code_in"])
    assert r["is_good"] == bool(f["warm_is_good"])
    ref = float(f["warm_loss"])
    assert abs(r["loss"] - ref) <= 0.05 * abs(ref)


def test_zhjd_query(gpu_decoder):
    f = golden("f7_secondary.npz")
    opt = _opt(gpu_decoder, S.KITTI_OPTIM, "KITTI")
    v = opt.compute_sdf_loss_objectpoint_zhjd(f["zhjd_pts"], f["code"])
    assert abs(v - float(f["zhjd_out"])) <= 2e-6


def test_full_size_batch_properties(gpu_decoder, oracle_dec):
    """BASELINE config 3 shape (16 KITTI objects x 2048 pts): all good, finite, and the
    first GN step of objects 0 and 11 matches the oracle's from the same state."""
    from oracle import dsr_oracle as O

    opt = _opt(gpu_decoder, S.KITTI_OPTIM, "KITTI")
    objs = [S.kitti_object(i) for i in range(16)]
    res, tr = opt.reconstruct_objects([(o.t_cam_obj, o.pts, o.rays, o.depth, None) for o in objs],
                                      trace=True)
    assert all(r["is_good"] for r in res)
    for r in res:
        assert np.isfinite(r["t_cam_obj"]).all() and np.isfinite(r["code"]).all()
        assert np.isfinite(r["loss"]) and r["loss"] > 0
    P = O.OptimParams.from_cfg(S.KITTI_OPTIM)
    for i in (0, 11):
        o, t = objs[i], tr[i]
        n_fg = o.depth.shape[0]
        dobs = np.concatenate([o.depth, np.zeros(o.rays.shape[0] - n_fg)]).astype(np.float32)
        tro, _, _ = O.gn_step(oracle_dec, P, t["t_obj_cam"][0], t["z"][0], o.pts, o.rays, dobs, n_fg)
        assert abs(int(t["k"][0]) - tro.k) <= 2 and abs(int(t["n_valid"][0]) - tro.n_valid) <= 2, i
        assert abs(t["sdf_loss"][0] - tro.sdf_loss) <= 5e-5 * abs(tro.sdf_loss), i
        flips = max(abs(int(t["k"][0]) - tro.k), 2)
        assert abs(t["render_loss"][0] - tro.render_loss) <= (1e-5 * abs(tro.render_loss)
                                                              + flips * 0.09 / tro.k), i
        assert rel(t["H"][0], tro.H) <= 5e-3, i
        assert step_err(t["dx"][0], tro.dx, tro.H) <= 2e-2, i


def test_pose_only_vs_golden(gpu_decoder, oracle_dec):
    """estimate_pose_cam_obj (optimizer.py:46-87) on device vs the reference (F7) and the oracle."""
    from oracle import dsr_oracle as O

    f = golden("f7_secondary.npz")
    opt = _opt(gpu_decoder, S.KITTI_OPTIM, "KITTI")
    T = opt.estimate_pose_cam_obj(f["t_se3"], float(f["scale"]), f["pts"], f["code"])
    ref = f["pose_only_out"]
    assert T.dtype == np.float32 and T.shape == (4, 4)
    assert np.abs(T - ref).max() <= 2e-5 * np.abs(ref).max(), np.abs(T - ref).max()
    To = O.estimate_pose_cam_obj(oracle_dec, O.OptimParams.from_cfg(S.KITTI_OPTIM), f["t_se3"],
                                 float(f["scale"]), f["pts"], f["code"])
    assert np.abs(T - To).max() <= 2e-5 * np.abs(To).max()


def test_pose_only_more_iterations_filters_inliers(gpu_decoder, oracle_dec):
    """With >5 pose-only iterations the e==4 inlier filter (optimizer.py:77-79) takes
    effect.  On the near-spherical synthetic shape yaw is unobservable (only the 1e-2
    damping holds it), so the object centre is compared, not the rotation."""
    from oracle import dsr_oracle as O

    cfg = dict(S.KITTI_OPTIM, pose_only_optim={"num_iterations": 7, "learning_rate": 1.0})
    opt = _opt(gpu_decoder, cfg, "KITTI")
    P = O.OptimParams.from_cfg(cfg)
    ob = S.kitti_object(11)
    T0 = ob.t_cam_obj.copy()
    s = float(np.cbrt(np.linalg.det(T0[:3, :3].astype(np.float64))))
    T0[:3, :3] /= s
    code = np.zeros(64, np.float32)
    T = opt.estimate_pose_cam_obj(T0, s, ob.pts[:700], code)
    To = O.estimate_pose_cam_obj(oracle_dec, P, T0, s, ob.pts[:700], code)
    assert np.isfinite(T).all()
    assert np.abs(T[:3, 3] - To[:3, 3]).max() <= 2e-2
    # every point an outlier after iteration 4 -> the reference divides by 0 points: NaN
    big = np.full(64, 3.0, np.float32)
    Tn = opt.estimate_pose_cam_obj(T0, s, ob.pts[:300], big)
    Tno = O.estimate_pose_cam_obj(oracle_dec, P, T0, s, ob.pts[:300], big)
    assert np.isnan(Tno).all() == np.isnan(Tn).all()


def _gpu_shard_worker(rank, world, port, q):
    import os
    import sys

    from conftest import PKG, REPO
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DSR_DEVICE="0")
    import torch.distributed as dist

    import synthetic as S
    from conftest import make_cfg
    from deep_sdf.workspace import decoder_from_state
    from reconstruct.optimizer import Optimizer
    from reconstruct.parallel import reconstruct_sharded

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS, device=0)
        opt = Optimizer(dec, make_cfg(S.REDWOOD_OPTIM, "Redwood"))
        objs = [(o.t_cam_obj, o.pts, o.rays, o.depth, None)
                for o in (S.redwood_object(i, n_pts=300) for i in range(6))]
        res = reconstruct_sharded(objs, opt.reconstruct_objects)
        if rank == 0:
            q.put([(r["is_good"], r["loss"], r["t_cam_obj"].tolist()) for r in res])
    finally:
        dist.destroy_process_group()


def test_sharded_two_ranks_on_device(gpu_decoder):
    """reconstruct_sharded with the real device solver (2 ranks sharing GPU 0, gloo for the
    gather here; RCCL on a multi-GPU node) == one batched call, bitwise."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gpu_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    opt = _opt(gpu_decoder, S.REDWOOD_OPTIM, "Redwood")
    ref = opt.reconstruct_objects([(o.t_cam_obj, o.pts, o.rays, o.depth, None)
                                   for o in (S.redwood_object(i, n_pts=300) for i in range(6))])
    for (good, loss, T), r in zip(got, ref):
        assert good and r["is_good"]
        assert np.float32(loss) == np.float32(r["loss"])
        assert np.array_equal(np.asarray(T, np.float32), r["t_cam_obj"])


def test_nan_propagation(gpu_decoder):
    """torch.relu propagates NaN (deep_sdf_decoder.py:103): a NaN point or code gives a NaN
    SDF, every other point of the same tile stays finite and unchanged."""
    from reconstruct.optimizer import sdf_eval

    rng = np.random.default_rng(9)
    x = rng.uniform(-0.8, 0.8, (100, 3)).astype(np.float32)
    z = (0.05 * rng.standard_normal(64)).astype(np.float32)
    y0 = sdf_eval(gpu_decoder, z, x)
    x2 = x.copy()
    x2[7, 1] = np.nan
    y1 = sdf_eval(gpu_decoder, z, x2)
    assert np.isnan(y1[7]) and np.isfinite(np.delete(y1, 7)).all()
    assert np.abs(np.delete(y1, 7) - np.delete(y0, 7)).max() <= 1e-6
    z2 = z.copy()
    z2[3] = np.nan
    assert np.isnan(sdf_eval(gpu_decoder, z2, x)).all()


def test_early_ray_termination_matches_full_decode(gpu_decoder, monkeypatch):
    """Render passes with early ray termination (k_sample_pass) vs decoding every in-ball
    sample (DSR_RENDER_PASSES=0): same N_valid and K, same step up to the per-tile
    split-fp16 scale (tiles are composed differently), and far fewer samples decoded.
    Exactness of the skip itself: tests/test_ert_cpu.py (bitwise, on the oracle)."""
    import ctypes

    import bench
    from reconstruct import _libdsr as L

    f = golden("f4_traj_kitti0.npz")
    one = dict(S.KITTI_OPTIM, joint_optim=dict(S.KITTI_OPTIM["joint_optim"], num_iterations=1))
    opt = _opt(gpu_decoder, one, "KITTI")
    n_it = int(f["n_iters_run"])
    objs = [(f["it_t_obj_cam"][e], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][e])
            for e in range(n_it)]
    out = {}
    # (the large-batch default, the small-batch default, a fine schedule)
    for spec in ("0", "8,12,16,20,24,32", "16,24", "4,5,6,7,8,9,10,11,12,14,16,20,24,28,32,40"):
        monkeypatch.setenv("DSR_TEST_HOOKS", "1")   # kernel switches are test hooks
        monkeypatch.setenv("DSR_RENDER_PASSES", spec)
        out[spec] = opt.reconstruct_objects(objs, trace=True, pose_is_obj_cam=True)
    full_res, full_tr = out["0"]
    for spec in list(out)[1:]:
        res, tr = out[spec]
        for e in range(n_it):
            assert res[e]["is_good"] == full_res[e]["is_good"]
            assert int(tr[e]["n_valid"][0]) == int(full_tr[e]["n_valid"][0])
            assert int(tr[e]["k"][0]) == int(full_tr[e]["k"][0]), (spec, e)
            assert abs(tr[e]["loss"][0] - full_tr[e]["loss"][0]) <= 1e-5 * abs(full_tr[e]["loss"][0])
            assert rel(tr[e]["H"][0], full_tr[e]["H"][0]) <= 1e-4
            assert step_err(tr[e]["dx"][0], full_tr[e]["dx"][0], full_tr[e]["H"][0]) <= 1e-3

    params = L.optim_params(one)
    pts = {}
    monkeypatch.setenv("DSR_STREAMS", "1")
    for spec in ("0", "8,12,16,20,24,32"):
        monkeypatch.setenv("DSR_TEST_HOOKS", "1")   # kernel switches are test hooks
        monkeypatch.setenv("DSR_RENDER_PASSES", spec)
        h, keep = bench.make_batch(gpu_decoder, params, 8, 1000)
        lib, ctx = gpu_decoder.ctx.lib, gpu_decoder.ctx
        try:
            ctx.check(lib.dsr_batch_run(h), "run")
            st = L.Stats()
            ctx.check(lib.dsr_batch_stats(h, ctypes.byref(st)), "stats")
            pts[spec] = (st.fwd_points, st.fwd_launches)
        finally:
            lib.dsr_batch_destroy(h)
    assert pts["0"][1] == 1 and pts["8,12,16,20,24,32"][1] == 7
    assert pts["8,12,16,20,24,32"][0] < 0.8 * pts["0"][0], pts


def test_mesh_extractor_matches_oracle_and_level_set(gpu_decoder):
    """MeshExtractor (optimizer.py:216-233) on device: grid decode + marching cubes equals
    the CPU restatement (oracle/dsr_mc.py) on the same decoded grid bit for bit, and the
    mesh is a closed, consistently oriented surface on the decoder's zero level set.
    (Against skimage's marching_cubes_lewiner, the reference's mesher: parity unpinned.)"""
    from oracle.dsr_mc import marching_cubes
    from reconstruct.optimizer import MeshExtractor, sdf_eval

    ex = MeshExtractor(gpu_decoder, 64, 48)
    for seed in range(2):
        code = (0.3 * np.random.default_rng(seed).standard_normal(64)).astype(np.float32)
        m = ex.extract_mesh_from_code(code)
        vol = ex.decode_grid(code).reshape(48, 48, 48)
        v, f = marching_cubes(vol)
        assert m.vertices.dtype == np.float32 and m.faces.dtype == np.int32
        assert np.array_equal(m.vertices, v) and np.array_equal(m.faces, f)
        assert f.shape[0] > 1000
        e = np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]])
        _, cnt = np.unique(np.sort(e, 1), axis=0, return_counts=True)
        assert set(cnt.tolist()) == {2} and np.unique(e, axis=0).shape[0] == e.shape[0]
        # the reference's voxel grid is sheared by its true-division indexing (create_voxel_grid,
        # utils.py:97-116: x = i + j/d + k/d^2, y = j + k/d voxels), marching cubes treats it as
        # regular: map each vertex back through that linear shear before evaluating the SDF
        h, d = 2.0 / 47, 48
        q = (v.astype(np.float64) + 1.0) / h
        shear = np.array([[1.0, 1.0 / d, 1.0 / d ** 2], [0.0, 1.0, 1.0 / d], [0.0, 0.0, 1.0]])
        s = sdf_eval(gpu_decoder, code, (h * q @ shear.T - 1.0).astype(np.float32))
        assert np.median(np.abs(s)) < 0.02 * h and np.abs(s).max() < 0.5 * h


def test_convert_sdf_voxels_to_mesh_on_a_caller_volume(gpu_decoder):
    """convert_sdf_voxels_to_mesh (utils.py:119-140) called on its own (dsr_mc_volume): on the
    MeshExtractor's decoded grid it returns exactly MeshExtractor's mesh; on analytic volumes
    (a sphere, a torus, as torch tensor and ndarray, odd sizes, a level other than 0, a volume
    without a crossing) exactly the CPU restatement's (oracle/dsr_mc.py).  (Against skimage's
    marching_cubes_lewiner: parity unpinned.)"""
    import torch

    from oracle.dsr_mc import marching_cubes
    from reconstruct.optimizer import MeshExtractor
    from reconstruct.utils import convert_sdf_voxels_to_mesh

    ex = MeshExtractor(gpu_decoder, 64, 40)
    code = (0.3 * np.random.default_rng(5).standard_normal(64)).astype(np.float32)
    m = ex.extract_mesh_from_code(code)
    v, f = convert_sdf_voxels_to_mesh(torch.from_numpy(ex.decode_grid(code).reshape(40, 40, 40)))
    assert v.dtype == np.float32 and f.dtype == np.int32
    assert np.array_equal(v, m.vertices) and np.array_equal(f, m.faces) and f.shape[0] > 500
    for d, level in ((33, 0.0), (17, 0.05), (2, 0.0)):
        g = np.linspace(-1.0, 1.0, d)
        x, y, z = np.meshgrid(g, g, g, indexing="ij")
        sphere = (np.sqrt(x * x + y * y + z * z) - 0.6).astype(np.float32)
        torus = (np.sqrt((np.sqrt(x * x + y * y) - 0.55) ** 2 + z * z) - 0.25).astype(np.float32)
        for vol in (sphere, torus):
            gv, gf = convert_sdf_voxels_to_mesh(vol, level=level)
            ov, of = marching_cubes(vol, level)
            assert np.array_equal(gv, ov) and np.array_equal(gf, of), (d, level)
    v, f = convert_sdf_voxels_to_mesh(np.ones((9, 9, 9), np.float32))
    assert v.shape == (0, 3) and f.shape == (0, 3)
    with pytest.raises(ValueError):
        convert_sdf_voxels_to_mesh(np.ones((4, 4, 5), np.float32))


def test_extract_map_objects_end_to_end(gpu_decoder, tmp_path):
    """MapObjects.txt -> objects/<id>.npy + .ply (extract_map_objects.py:46-63) on device."""
    from reconstruct.map_objects import extract_map_objects, write_map_objects
    from reconstruct.optimizer import MeshExtractor
    from reconstruct.utils import read_mesh_ply

    rng = np.random.default_rng(3)
    objs = [(i, np.eye(4, dtype=np.float32), (0.2 * rng.standard_normal(64)).astype(np.float32))
            for i in (4, 9)]
    write_map_objects(str(tmp_path / "MapObjects.txt"), objs)
    ex = MeshExtractor(gpu_decoder, 64, 32)
    assert extract_map_objects(str(tmp_path), ex) == [4, 9]
    for oid, _, code in objs:
        pose = np.load(tmp_path / "objects" / f"{oid}.npy")
        assert np.array_equal(pose, np.eye(4))
        v, f = read_mesh_ply(str(tmp_path / "objects" / f"{oid}.ply"))
        m = ex.extract_mesh_from_code(np.asarray([float(f"{x:.9f}") for x in code], np.float32))
        assert np.array_equal(v, m.vertices) and np.array_equal(f, m.faces) and f.shape[0] > 100


def test_graph_replay_bitwise(gpu_decoder, monkeypatch):
    """DSR_GRAPH=1: a re-run batch is captured into a hipGraph (2nd run) and replayed (3rd):
    results and per-iteration counters identical to the eager first run."""
    import ctypes

    import bench
    from reconstruct import _libdsr as L

    lib, ctx = gpu_decoder.ctx.lib, gpu_decoder.ctx
    params = L.optim_params(dict(S.REDWOOD_OPTIM))
    for graph in ("1", "0"):
        monkeypatch.setenv("DSR_GRAPH", graph)
        h, keep = bench.make_batch(gpu_decoder, params, 6, 4000)
        try:
            sig = []
            for _ in range(3):
                outs = (L.ObjectOut * 6)()
                ctx.check(lib.dsr_batch_run(h), "run")
                ctx.check(lib.dsr_batch_download(h, outs), "download")
                st = L.Stats()
                ctx.check(lib.dsr_batch_stats(h, ctypes.byref(st)), "stats")
                assert st.total_ms > 0
                replay = graph == "1" and len(sig) > 0
                assert (st.fwd_launches == 0) if replay else (st.fwd_ms > 0 and st.jac_ms > 0)
                sig.append((np.array([list(o.t_cam_obj) + list(o.code) + [o.loss, o.is_good] for o in outs],
                                     np.float32), st.fwd_points, st.jac_points, st.inball_points))
            for s in sig[1:]:
                assert np.array_equal(s[0], sig[0][0]) and s[1:] == sig[0][1:]
        finally:
            lib.dsr_batch_destroy(h)


@pytest.mark.parametrize("streams", ["1", "2"])
def test_graph_replays_never_return_stale_records(gpu_decoder, monkeypatch, streams):
    """Every replay poisons the out-records on the stream before its hipGraphLaunch and the
    graph's k_finalize rewrites them; 150 replays, each downloaded at once, must all equal the
    eager run — a download ordered before the graph's last kernel (or the poison after it)
    would return the poison bytes.  ``streams`` 2: the captured two-group fork / join (round 3
    saw an event recorded after a per-group graph launch fail to order later work, DESIGN
    §3.5); 1: the graph mode's default one-group batch."""
    from reconstruct import _libdsr as L

    import bench

    lib, ctx = gpu_decoder.ctx.lib, gpu_decoder.ctx
    params = L.optim_params(dict(S.REDWOOD_OPTIM, joint_optim=dict(S.REDWOOD_OPTIM["joint_optim"],
                                                                    num_iterations=2)))
    monkeypatch.setenv("DSR_STREAMS", streams)
    ref = None
    for graph in ("0", "1"):
        monkeypatch.setenv("DSR_GRAPH", graph)
        h, keep = bench.make_batch(gpu_decoder, params, 8, 4100)
        try:
            for r in range(150 if graph == "1" else 1):
                outs = (L.ObjectOut * 8)()
                ctx.check(lib.dsr_batch_run(h), "run")
                ctx.check(lib.dsr_batch_download(h, outs), "download")
                if ref is None:
                    ref = bytes(outs)
                    assert all(o.is_good in (0, 1) for o in outs)
                assert bytes(outs) == ref, f"replay {r} differs"
        finally:
            lib.dsr_batch_destroy(h)


def test_lite_pass_matches_exact_decode(gpu_decoder, monkeypatch):
    """The one-product classification pass + exact re-decode of the band (dsr_mlp_lite.hpp)
    vs decoding every sample exactly (DSR_LITE=0): same N_valid, K and step; and the pass's
    own error monitor stays far inside the margin it calibrates."""
    import ctypes

    import bench
    from reconstruct import _libdsr as L

    f = golden("f4_traj_kitti0.npz")
    one = dict(S.KITTI_OPTIM, joint_optim=dict(S.KITTI_OPTIM["joint_optim"], num_iterations=1))
    opt = _opt(gpu_decoder, one, "KITTI")
    n_it = int(f["n_iters_run"])
    objs = [(f["it_t_obj_cam"][e], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][e])
            for e in range(n_it)]
    out = {}
    # exact decode | lite + exact band, Jacobian re-forwards render points | ... masks kept
    for lite, keep in (("0", "1"), ("1", "0"), ("1", "1")):
        monkeypatch.setenv("DSR_LITE", lite)
        monkeypatch.setenv("DSR_TEST_HOOKS", "1")   # kernel switches are test hooks
        monkeypatch.setenv("DSR_KEEP_MASKS", keep)
        out[lite + keep] = opt.reconstruct_objects(objs, trace=True, pose_is_obj_cam=True)
    r0, t0 = out["01"]
    for key in ("10", "11"):
        r1, t1 = out[key]
        for e in range(n_it):
            assert r1[e]["is_good"] == r0[e]["is_good"]
            assert int(t1[e]["n_valid"][0]) == int(t0[e]["n_valid"][0])
            assert int(t1[e]["k"][0]) == int(t0[e]["k"][0]), (key, e)
            assert abs(t1[e]["loss"][0] - t0[e]["loss"][0]) <= 1e-5 * abs(t0[e]["loss"][0])
            assert rel(t1[e]["H"][0], t0[e]["H"][0]) <= 1e-4, (key, e)
            assert step_err(t1[e]["dx"][0], t0[e]["dx"][0], t0[e]["H"][0]) <= 1e-3, (key, e)
    monkeypatch.delenv("DSR_KEEP_MASKS")

    monkeypatch.setenv("DSR_LITE", "1")
    lib, ctx = gpu_decoder.ctx.lib, gpu_decoder.ctx
    h, keep = bench.make_batch(gpu_decoder, L.optim_params(S.KITTI_OPTIM), 8, 1000)
    try:
        ctx.check(lib.dsr_batch_run(h), "run")
        st = L.Stats()
        ctx.check(lib.dsr_batch_stats(h, ctypes.byref(st)), "stats")
    finally:
        lib.dsr_batch_destroy(h)
    assert st.lite == 1 and st.refine_points > 0 and st.refine_launches > 0
    # calibrated margin max(0.002, 4 x the largest observed error), well inside th = 0.01
    assert 0.0 < st.lite_max_err < 1e-3
    assert 0.002 - 1e-7 <= st.lite_min_margin <= max(0.002, 4 * st.lite_max_err) + 1e-7


@pytest.mark.gpu
def test_refine_stops_at_ray_termination(gpu_decoder, monkeypatch):
    """k_refine_scan skips band samples behind a ray's first certainly-full sample (their
    transmittance is exactly 0): results bitwise those of refining every band sample
    (DSR_REFINE_ALL=1), with fewer samples re-decoded."""
    import ctypes

    import bench
    from reconstruct import _libdsr as L

    lib, ctx = gpu_decoder.ctx.lib, gpu_decoder.ctx
    monkeypatch.setenv("DSR_LITE", "1")
    sig = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("DSR_TEST_HOOKS", "1")   # kernel switches are test hooks
        monkeypatch.setenv("DSR_REFINE_ALL", mode)
        h, keep = bench.make_batch(gpu_decoder, L.optim_params(S.KITTI_OPTIM), 8, 1000)
        try:
            outs = (L.ObjectOut * 8)()
            ctx.check(lib.dsr_batch_run(h), "run")
            ctx.check(lib.dsr_batch_download(h, outs), "download")
            st = L.Stats()
            ctx.check(lib.dsr_batch_stats(h, ctypes.byref(st)), "stats")
            rec = np.array([list(o.t_cam_obj) + list(o.code) + [o.loss, o.is_good, o.iters_done] for o in outs],
                           np.float32)
            sig[mode] = (rec, st.refine_points, st.fwd_points, st.jac_points)
        finally:
            lib.dsr_batch_destroy(h)
    assert np.array_equal(sig["0"][0], sig["1"][0])
    assert sig["0"][2:] == sig["1"][2:]
    assert 0 < sig["0"][1] < sig["1"][1]


@pytest.mark.gpu
def test_lite_staggered_groups_bitwise(gpu_decoder, monkeypatch):
    """The staggered-group lite kernel (default DSR_LITE_VARIANT=1496: LDS event counters
    instead of block barriers, dsr_mlp_lite.hpp: k_mlp_fwd_lite_st) gives the same lite values
    whatever the stagger lag (0: B may start each GEMM at once, 7: half a GEMM behind) — a
    race on the LDS image would change values, classes and counts — and equals the unswizzled
    variant 472 bitwise; no block's bounded event wait expires (dsr_stats.lite_broken_blocks).
    (Round 2 tested the scaled-epilogue variant 216 against the barrier kernel 88 here; 216
    is no longer in the shipped library)"""
    import ctypes

    import bench
    from reconstruct import _libdsr as L

    lib, ctx = gpu_decoder.ctx.lib, gpu_decoder.ctx
    monkeypatch.setenv("DSR_LITE", "1")
    sig = {}
    for v, lag in (("1496", "4"), ("1496", "0"), ("1496", "7"), ("472", "4")):
        monkeypatch.setenv("DSR_TEST_HOOKS", "1")   # kernel switches are test hooks
        monkeypatch.setenv("DSR_LITE_VARIANT", v)
        monkeypatch.setenv("DSR_LITE_LAG", lag)
        h, keep = bench.make_batch(gpu_decoder, L.optim_params(S.KITTI_OPTIM), 8, 1000)
        try:
            outs = (L.ObjectOut * 8)()
            ctx.check(lib.dsr_batch_run(h), "run")
            ctx.check(lib.dsr_batch_download(h, outs), "download")
            st = L.Stats()
            ctx.check(lib.dsr_batch_stats(h, ctypes.byref(st)), "stats")
            rec = np.array([list(o.t_cam_obj) + list(o.code) + [o.loss, o.is_good, o.iters_done] for o in outs],
                           np.float32)
            sig[(v, lag)] = (rec, st.fwd_points, st.refine_points, st.jac_points)
            assert st.lite_broken_blocks == 0, (v, lag, L.lite_diag(lib, h))
        finally:
            lib.dsr_batch_destroy(h)
    ref = sig[("1496", "4")]
    for k, s in sig.items():
        assert np.array_equal(s[0].view(np.uint32), ref[0].view(np.uint32)), k
        assert s[1:] == ref[1:], k


@pytest.mark.gpu
def test_lite_broken_block_falls_back_to_exact(gpu_decoder, monkeypatch):
    """A staggered lite block whose event wait times out marks itself broken and sends every
    sample it classifies to the exact pass.  Forced on every block (DSR_LITE_BREAK=1), all
    samples are re-decoded exactly and no ray terminates early on a lite value: results
    bitwise those of the exact path (DSR_LITE=0; early ray termination is exact)."""
    import ctypes

    import bench
    from reconstruct import _libdsr as L

    lib, ctx = gpu_decoder.ctx.lib, gpu_decoder.ctx
    sig = {}
    monkeypatch.setenv("DSR_TEST_HOOKS", "1")
    for mode in ("exact", "broken"):
        monkeypatch.setenv("DSR_LITE", "0" if mode == "exact" else "1")
        monkeypatch.setenv("DSR_LITE_BREAK", "1" if mode == "broken" else "0")
        h, keep = bench.make_batch(gpu_decoder, L.optim_params(S.KITTI_OPTIM), 4, 1000)
        try:
            outs = (L.ObjectOut * 4)()
            ctx.check(lib.dsr_batch_run(h), "run")
            ctx.check(lib.dsr_batch_download(h, outs), "download")
            st = L.Stats()
            ctx.check(lib.dsr_batch_stats(h, ctypes.byref(st)), "stats")
            rec = np.array([list(o.t_cam_obj) + list(o.code) + [o.loss, o.is_good, o.iters_done] for o in outs],
                           np.float32)
            sig[mode] = (rec, st.jac_points, st.refine_points, st.fwd_points)
            if mode == "broken":      # every started block counted as broken (dsr_stats)
                assert st.test_hooks == 1 and st.lite_broken_blocks > 0
        finally:
            lib.dsr_batch_destroy(h)
    assert np.array_equal(sig["broken"][0].view(np.uint32), sig["exact"][0].view(np.uint32))
    assert sig["broken"][1] == sig["exact"][1]
    assert sig["broken"][2] == sig["broken"][3] > 0      # every lite-classified sample refined


def test_large_batch_tile_tables(gpu_decoder, monkeypatch):
    """Batches of more than 1024 objects: the block-scan tile tables (k_tiles_fwd/_jac,
    tile_scan) cross their 1024-object chunks; objects on both sides of the boundary match
    their one-by-one runs bitwise."""
    monkeypatch.setenv("DSR_STREAMS", "1")
    opt = _opt(gpu_decoder, dict(S.REDWOOD_OPTIM, joint_optim=dict(S.REDWOOD_OPTIM["joint_optim"],
                                                                    num_iterations=2)), "Redwood")
    objs = []
    for i in range(1100):
        o = S.make_object(5000 + i, n_pts=40 + (i % 7), n_bg=8, scale=1.0, tz=3.0, upright=False)
        objs.append((o.t_cam_obj, o.pts, o.rays, o.depth, None))
    batch, tr = opt.reconstruct_objects(objs, trace=True)
    for i in (0, 1, 1023, 1024, 1025, 1099):
        single, tr1 = opt.reconstruct_objects([objs[i]], trace=True)
        assert batch[i]["is_good"] == single[0]["is_good"], i
        assert batch[i]["loss"] == single[0]["loss"], i
        for key in ("H", "b", "n_valid", "k"):
            assert np.array_equal(tr[i][key], tr1[0][key]), (i, key)


@pytest.mark.gpu
def test_surface_forward_in_exact_pass_bitwise(gpu_decoder, monkeypatch):
    """Small batches run the surface points' forward in the exact pass and keep their ReLU
    masks (MaskArgs.pts), so the Jacobian kernel only chains backward passes; the forward
    is the same split-fp16 arithmetic on the same 64-point tiles, so every output and count
    is bitwise that of the Jacobian kernel forwarding them itself (DSR_SURFACE_EXACT=0)."""
    import ctypes

    import bench
    from reconstruct import _libdsr as L

    lib, ctx = gpu_decoder.ctx.lib, gpu_decoder.ctx
    monkeypatch.setenv("DSR_LITE", "1")
    sig = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("DSR_TEST_HOOKS", "1")   # kernel switches are test hooks
        monkeypatch.setenv("DSR_SURFACE_EXACT", mode)
        h, keep = bench.make_batch(gpu_decoder, L.optim_params(S.KITTI_OPTIM), 6, 1000)
        try:
            outs = (L.ObjectOut * 6)()
            ctx.check(lib.dsr_batch_run(h), "run")
            ctx.check(lib.dsr_batch_download(h, outs), "download")
            st = L.Stats()
            ctx.check(lib.dsr_batch_stats(h, ctypes.byref(st)), "stats")
            rec = np.array([list(o.t_cam_obj) + list(o.code) + [o.loss, o.is_good, o.iters_done] for o in outs],
                           np.float32)
            sig[mode] = (rec, st.fwd_points, st.refine_points, st.jac_surface_points, st.jac_render_points)
            assert st.surface_in_exact == int(mode)
        finally:
            lib.dsr_batch_destroy(h)
    assert np.array_equal(sig["0"][0].view(np.uint32), sig["1"][0].view(np.uint32))
    assert sig["0"][1:] == sig["1"][1:]


@pytest.mark.gpu
def test_ray_chunk_boundaries_vs_oracle(gpu_decoder, oracle_dec):
    """The render and refine kernels run one workgroup per 128 rays of an object (ray
    chunks) and stitch the chunks' ordered outputs together: objects whose
    ray counts sit on and around chunk boundaries (128, 129, 256, 257, 383 rays), batched
    together, each give the oracle's first GN step from the same state."""
    from oracle import dsr_oracle as O

    opt = _opt(gpu_decoder, dict(S.REDWOOD_OPTIM, joint_optim=dict(S.REDWOOD_OPTIM["joint_optim"],
                                                                     num_iterations=1)), "Redwood")
    shapes = [(100, 28), (100, 29), (200, 56), (200, 57), (300, 83)]
    obs = [S.make_object(900 + i, n_pts=n, n_bg=b, scale=1.0, tz=3.0, upright=False)
           for i, (n, b) in enumerate(shapes)]
    assert [o.rays.shape[0] for o in obs] == [128, 129, 256, 257, 383]
    res, tr = opt.reconstruct_objects([(o.t_cam_obj, o.pts, o.rays, o.depth, None) for o in obs], trace=True)
    P = O.OptimParams.from_cfg(S.REDWOOD_OPTIM)
    for i, o in enumerate(obs):
        assert res[i]["is_good"], (i, res[i])
        t = tr[i]
        n_fg = o.depth.shape[0]
        dobs = np.concatenate([o.depth, np.zeros(o.rays.shape[0] - n_fg)]).astype(np.float32)
        tro, _, _ = O.gn_step(oracle_dec, P, t["t_obj_cam"][0], t["z"][0], o.pts, o.rays, dobs, n_fg)
        dk = abs(int(t["k"][0]) - tro.k)
        assert dk <= 2 and abs(int(t["n_valid"][0]) - tro.n_valid) <= 2, i
        assert abs(t["sdf_loss"][0] - tro.sdf_loss) <= 5e-5 * abs(tro.sdf_loss), i
        assert abs(t["render_loss"][0] - tro.render_loss) <= (1e-5 * abs(tro.render_loss)
                                                              + max(dk, 2) * 0.09 / tro.k), i
        assert rel(t["H"][0], tro.H) <= 5e-3, i


@pytest.mark.gpu
@pytest.mark.parametrize("m", [17, 32, 64])
def test_depth_sample_counts_vs_oracle(gpu_decoder, oracle_dec, m, monkeypatch):
    """num_depth_samples (configs' `num_depth_samples`, optimizer.py:126) other than 50:
    odd, small, and the largest supported (64: every lane of the refine scan, the largest
    render LDS rows) — the first GN step of a small batch vs the oracle's; and the same batch
    as one object group (the render passes over ray chunks, rows of M samples at any 4-byte
    alignment in the render staging) bitwise equal to the default grouping."""
    from oracle import dsr_oracle as O

    optim = dict(S.REDWOOD_OPTIM, num_depth_samples=m,
                 joint_optim=dict(S.REDWOOD_OPTIM["joint_optim"], num_iterations=1))
    opt = _opt(gpu_decoder, optim, "Redwood")
    obs = [S.redwood_object(60 + i, n_pts=300) for i in range(3)]
    objs = [(o.t_cam_obj, o.pts, o.rays, o.depth, None) for o in obs]
    res, tr = opt.reconstruct_objects(objs, trace=True)
    monkeypatch.setenv("DSR_STREAMS", "1")
    res1, tr1 = opt.reconstruct_objects(objs, trace=True)
    for i in range(len(objs)):
        assert res1[i]["loss"] == res[i]["loss"], (m, i)
        for key in ("H", "b", "n_valid", "k", "n_decoded", "n_refined"):
            assert np.array_equal(tr1[i][key], tr[i][key]), (m, i, key)
    P = O.OptimParams.from_cfg(optim)
    assert P.num_depth_samples == m
    for i, o in enumerate(obs):
        assert res[i]["is_good"], (i, res[i])
        t = tr[i]
        n_fg = o.depth.shape[0]
        dobs = np.concatenate([o.depth, np.zeros(o.rays.shape[0] - n_fg)]).astype(np.float32)
        tro, _, _ = O.gn_step(oracle_dec, P, t["t_obj_cam"][0], t["z"][0], o.pts, o.rays, dobs, n_fg)
        dk = abs(int(t["k"][0]) - tro.k)
        assert dk <= 2 and abs(int(t["n_valid"][0]) - tro.n_valid) <= 2, (m, i)
        assert abs(t["sdf_loss"][0] - tro.sdf_loss) <= 5e-5 * abs(tro.sdf_loss), (m, i)
        assert abs(t["render_loss"][0] - tro.render_loss) <= (1e-5 * abs(tro.render_loss)
                                                              + max(dk, 2) * 0.09 / tro.k), (m, i)
        assert rel(t["H"][0], tro.H) <= 5e-3, (m, i)
