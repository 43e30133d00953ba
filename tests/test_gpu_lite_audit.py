"""The lite classification pass is guarded, not trusted.

The one-product fp16 pass (dsr_mlp_lite.hpp) only has to tell, for every ray sample,
whether its sdf is certainly >= th (empty), certainly <= -th (full) or possibly in the
band (loss_utils.py:40-48, loss.py:101-102); the band is re-decoded exactly.  Its
margin calibrates itself from measured errors, and every iteration an AUDIT re-decodes
exactly the out-of-band samples within th + 2*margin plus a hashed 1/128 of all others
(dsr_dev.hpp: lite_flag).  Their error feeds the calibration; a class disagreement on
any of them discards that object's iteration and redoes it, and the rest of the run,
with every sample decoded exactly (k_solve, k_iter_begin).

These tests (1) force violations with a deterministic perturbation of every lite value
(DSR_LITE_PERTURB, a test hook the library honours only under DSR_TEST_HOOKS=1) and show the guard fires and the results equal exact decoding
(DSR_LITE=0) at the teacher-forced tolerances; (2) check later iterations — where the
margin has calibrated down to max(0.002, 4 x the observed error) — against exact decoding from the same
state, on the bench decoder and on a decoder with larger hidden weights (larger
activations, larger fp16 error).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import synthetic as S
from conftest import golden, make_cfg

pytestmark = pytest.mark.gpu


def _opt(dec, optim, data_type="KITTI", iters=None):
    from reconstruct.optimizer import Optimizer

    if iters is not None:
        optim = dict(optim, joint_optim=dict(optim["joint_optim"], num_iterations=iters))
    return Optimizer(dec, make_cfg(optim, data_type))


def rel(a, b):
    return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


def batch_stats(opt, objects, pose_is_obj_cam=False):
    """Run ``objects`` through the resident-batch API; return (outs, dsr_stats)."""
    from reconstruct import _libdsr as L

    keep = []
    n = len(objects)
    ins = (L.ObjectIn * n)()
    for i, ob in enumerate(objects):
        ins[i] = opt._object_in(*ob[:4], ob[4] if len(ob) > 4 else None, keep, pose_is_obj_cam)
    ctx = opt._ctx
    h = C.c_void_p()
    ctx.check(ctx.lib.dsr_batch_create(ctx.handle, opt.decoder.handle, C.byref(opt.params), n, ins,
                                       C.byref(h)), "create")
    try:
        outs = (L.ObjectOut * n)()
        ctx.check(ctx.lib.dsr_batch_run(h), "run")
        ctx.check(ctx.lib.dsr_batch_download(h, outs), "download")
        st = L.Stats()
        ctx.check(ctx.lib.dsr_batch_stats(h, C.byref(st)), "stats")
    finally:
        ctx.lib.dsr_batch_destroy(h)
    return outs, st


def assert_same_step(t1, t0, e1=0, e0=0, what=""):
    """One GN iteration's terms agree like the lite-vs-exact A/B of test_gpu_parity."""
    assert int(t1["n_valid"][e1]) == int(t0["n_valid"][e0]), what
    assert int(t1["k"][e1]) == int(t0["k"][e0]), what
    assert abs(t1["loss"][e1] - t0["loss"][e0]) <= 1e-5 * abs(t0["loss"][e0]), what
    assert rel(t1["H"][e1], t0["H"][e0]) <= 1e-4, what
    d = np.asarray(t1["dx"][e1], np.float64) - t0["dx"][e0]
    H = np.asarray(t0["H"][e0], np.float64)
    dx0 = np.asarray(t0["dx"][e0], np.float64)
    assert np.sqrt(max(d @ H @ d, 0) / max(dx0 @ H @ dx0, 1e-300)) <= 1e-3, what


def test_audit_guard_fires_and_redoes_exactly(gpu_decoder, monkeypatch):
    f = golden("f4_traj_kitti0.npz")
    opt = _opt(gpu_decoder, S.KITTI_OPTIM, iters=1)
    objs = [(f["it_t_obj_cam"][e], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][e])
            for e in (0, 4, 9)]
    monkeypatch.setenv("DSR_LITE", "0")
    r0, t0 = opt.reconstruct_objects(objs, trace=True, pose_is_obj_cam=True)
    monkeypatch.setenv("DSR_LITE", "1")
    # every lite value off by +-0.015: band samples (|sdf| < th = 0.01) that leave the band
    # (th + m, first-iteration margin m = 0.01) all land in the audit shell th+m..th+2m, so
    # every object sees violations
    monkeypatch.setenv("DSR_LITE_PERTURB", "0.015")
    monkeypatch.setenv("DSR_TEST_HOOKS", "1")
    outs, st = batch_stats(opt, objs, pose_is_obj_cam=True)
    assert st.test_hooks == 1
    assert st.lite == 1 and st.audit_points > 0
    assert st.lite_audit_violations > 0
    assert st.lite_redo_objects == len(objs)
    assert all(outs[i].is_good and outs[i].iters_done == 1 for i in range(len(objs)))
    r1, t1 = opt.reconstruct_objects(objs, trace=True, pose_is_obj_cam=True)
    for i in range(len(objs)):
        assert r1[i]["is_good"] and r0[i]["is_good"]
        assert_same_step(t1[i], t0[i], what=f"object {i}")
    # without the audit the same perturbation silently changes the render set
    monkeypatch.setenv("DSR_LITE_AUDIT", "0")
    r2, t2 = opt.reconstruct_objects(objs, trace=True, pose_is_obj_cam=True)
    assert any(int(t2[i]["k"][0]) != int(t0[i]["k"][0]) for i in range(len(objs)))


def test_audit_shell_catches_with_certainty(gpu_decoder, monkeypatch):
    """The certain part of the audit alone (hashed share 2^-24: practically none): lite values
    perturbed by +-0.015 push band samples (|sdf| < th = 0.01, first-iteration margin m = 0.01)
    into th+m..th+2m, the shell, which is re-decoded whatever the hash says — every object sees
    violations and is redone.  With the shell off (DSR_LITE_SHELL=0, the shipped behaviour
    before round 3's fix: the shell sat on the band edge) the same run audits almost nothing."""
    f = golden("f4_traj_kitti0.npz")
    opt = _opt(gpu_decoder, S.KITTI_OPTIM, iters=1)
    objs = [(f["it_t_obj_cam"][e], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][e])
            for e in (0, 4, 9)]
    monkeypatch.setenv("DSR_LITE", "1")
    monkeypatch.setenv("DSR_TEST_HOOKS", "1")
    monkeypatch.setenv("DSR_LITE_PERTURB", "0.015")
    monkeypatch.setenv("DSR_LITE_AUDIT_LOG2", "24")
    outs, st = batch_stats(opt, objs, pose_is_obj_cam=True)
    assert st.lite_audit_violations > 0 and st.lite_redo_objects == len(objs)
    assert all(outs[i].is_good and outs[i].iters_done == 1 for i in range(len(objs)))
    monkeypatch.setenv("DSR_LITE_SHELL", "0")
    _, st0 = batch_stats(opt, objs, pose_is_obj_cam=True)
    assert st0.audit_points < 0.01 * st.audit_points, (st0.audit_points, st.audit_points)
    assert st0.lite_audit_violations < st.lite_audit_violations


def test_audit_everything_mode(gpu_decoder, monkeypatch):
    """DSR_LITE_AUDIT_LOG2=0 (tools/lite_audit_all.py): every sample the lite pass decoded up to
    its ray's first certainly-full one is re-decoded exactly — band samples as band, all others
    as audits — and no class differs.  (Samples behind that one, decoded because they share its
    pass window, are not: transmittance is exactly 0 there, §3.3; ~9% of the lite samples.)"""
    monkeypatch.setenv("DSR_LITE", "1")
    monkeypatch.setenv("DSR_TEST_HOOKS", "1")
    monkeypatch.setenv("DSR_LITE_AUDIT_LOG2", "0")
    opt = _opt(gpu_decoder, S.KITTI_OPTIM, iters=3)
    objs = [S.kitti_object(i) for i in range(4)]
    outs, st = batch_stats(opt, [(o.t_cam_obj, o.pts, o.rays, o.depth, None) for o in objs])
    assert all(outs[i].is_good for i in range(len(objs)))
    assert st.lite_audit_violations == 0 and st.lite_redo_objects == 0
    assert 0.8 * st.fwd_points <= st.refine_points <= st.fwd_points, (st.refine_points, st.fwd_points)
    assert st.audit_points > 0.5 * st.fwd_points


def test_audit_quiet_and_cheap_on_the_bench_workload(gpu_decoder, monkeypatch):
    """Unperturbed: no violation, the audit re-decodes a bounded share of the samples."""
    monkeypatch.setenv("DSR_LITE", "1")
    opt = _opt(gpu_decoder, S.KITTI_OPTIM)
    objs = [S.kitti_object(i) for i in range(8)]
    outs, st = batch_stats(opt, [(o.t_cam_obj, o.pts, o.rays, o.depth, None) for o in objs])
    assert st.lite_audit_violations == 0 and st.lite_redo_objects == 0
    # the default staggered kernel never hit a bounded event wait
    assert st.lite_broken_blocks == 0 and st.test_hooks == 0
    assert st.audit_points > 0
    assert st.audit_points <= 0.1 * st.fwd_points, (st.audit_points, st.fwd_points)
    # margin = max(0.002, 4 x the object's largest observed error), well inside th = 0.01
    assert 0.0 < st.lite_max_err < 1e-3
    assert 0.002 - 1e-7 <= st.lite_min_margin <= max(0.002, 4 * st.lite_max_err) + 1e-7


@pytest.mark.parametrize("gain", [2.45, 3.2], ids=["bench_decoder", "larger_weights"])
def test_calibrated_margin_iterations_match_exact(gain, monkeypatch):
    """Iterations 1.. of a lite run (calibrated margin) vs exact decoding from that state."""
    from deep_sdf.workspace import decoder_from_state

    if gain == 2.45:
        state = S.make_decoder(1234)
    else:
        state = S.fit_last_layer_to_sphere(S.make_decoder_state(1234, hidden_gain=gain))
    dec = decoder_from_state(state, S.DEFAULT_SPECS)
    opt = _opt(dec, S.KITTI_OPTIM, iters=4)
    one = _opt(dec, S.KITTI_OPTIM, iters=1)
    objs = [S.kitti_object(i) for i in (0, 3)]
    monkeypatch.setenv("DSR_LITE", "1")
    res, tr = opt.reconstruct_objects([(o.t_cam_obj, o.pts, o.rays, o.depth, None) for o in objs],
                                      trace=True)
    outs, st = batch_stats(opt, [(o.t_cam_obj, o.pts, o.rays, o.depth, None) for o in objs])
    assert st.lite_audit_violations == 0, st.lite_audit_violations
    for i, o in enumerate(objs):
        assert res[i]["is_good"]
        states = [(tr[i]["t_obj_cam"][e], o.pts, o.rays, o.depth, tr[i]["z"][e]) for e in (1, 2, 3)]
        monkeypatch.setenv("DSR_LITE", "0")
        r0, t0 = one.reconstruct_objects(states, trace=True, pose_is_obj_cam=True)
        monkeypatch.setenv("DSR_LITE", "1")
        for j, e in enumerate((1, 2, 3)):
            assert_same_step(tr[i], t0[j], e1=e, e0=0, what=f"gain {gain} object {i} iteration {e}")


def test_test_hooks_ignored_without_the_gate(gpu_decoder, monkeypatch):
    """DSR_LITE_PERTURB / DSR_LITE_BREAK change nothing unless DSR_TEST_HOOKS=1 (a stray
    variable cannot alter a production run), and dsr_stats reports the gate."""
    f = golden("f4_traj_kitti0.npz")
    opt = _opt(gpu_decoder, S.KITTI_OPTIM, iters=1)
    objs = [(f["it_t_obj_cam"][0], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][0])]
    monkeypatch.setenv("DSR_LITE", "1")
    monkeypatch.delenv("DSR_TEST_HOOKS", raising=False)
    ref, st0 = batch_stats(opt, objs, pose_is_obj_cam=True)
    monkeypatch.setenv("DSR_LITE_PERTURB", "0.015")
    monkeypatch.setenv("DSR_LITE_BREAK", "1")
    outs, st = batch_stats(opt, objs, pose_is_obj_cam=True)
    assert st.test_hooks == 0 and st0.test_hooks == 0
    assert st.lite_audit_violations == 0 and st.lite_broken_blocks == 0
    assert st.refine_points == st0.refine_points < st.fwd_points
    assert bytes(outs) == bytes(ref)


GUARD_KNOBS = {"DSR_LITE_AUDIT": "0", "DSR_LITE_SHELL": "0", "DSR_LITE_AUDIT_LOG2": "24",
               "DSR_LITE_MARGIN": "0.05", "DSR_LITE_FLOOR": "0.0001", "DSR_LITE_SAFETY": "0.5"}


def test_guard_settings_ignored_without_the_gate(gpu_decoder, monkeypatch):
    """The lite pass's guard is part of the product: without
    DSR_TEST_HOOKS=1 the variables that would switch the audit off, drop its certain shell, thin
    its hashed share or move the margin change nothing — bytes equal — and dsr_stats reports the
    settings the batch actually ran with."""
    f = golden("f4_traj_kitti0.npz")
    opt = _opt(gpu_decoder, S.KITTI_OPTIM, iters=3)
    objs = [(f["it_t_obj_cam"][e], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][e]) for e in (0, 4)]
    monkeypatch.setenv("DSR_LITE", "1")
    monkeypatch.delenv("DSR_TEST_HOOKS", raising=False)
    for k in GUARD_KNOBS:
        monkeypatch.delenv(k, raising=False)
    ref, st0 = batch_stats(opt, objs, pose_is_obj_cam=True)
    for k, v in GUARD_KNOBS.items():
        monkeypatch.setenv(k, v)
    outs, st = batch_stats(opt, objs, pose_is_obj_cam=True)
    assert bytes(outs) == bytes(ref)
    for s in (st0, st):
        assert s.test_hooks == 0 and s.lite == 1 and s.lite_eligible == 1
        assert s.audit == 1 and s.audit_shell == 1.0 and s.audit_log2 == 7
        assert abs(s.lite_margin0 - 0.01) < 1e-7 and abs(s.lite_floor - 0.002) < 1e-7 and s.lite_safety == 4.0
    assert st.audit_points == st0.audit_points > 0
    # under the gate the same variables do take effect (the survey / test paths)
    monkeypatch.setenv("DSR_TEST_HOOKS", "1")
    _, sh = batch_stats(opt, objs, pose_is_obj_cam=True)
    assert sh.test_hooks == 1 and sh.audit == 0 and sh.audit_points == 0 and sh.audit_shell == 0.0
    assert abs(sh.lite_floor - 1e-4) < 1e-9 and sh.lite_safety == 0.5


def test_bench_decoder_qualifies_for_the_lite_pass(gpu_decoder):
    """dsr_decoder_load's probe (65,536 points in the unit ball x 4 codes, lite vs exact): the
    bench decoder's lite error stays far inside half the distance to a class boundary."""
    info = gpu_decoder.info
    assert info["lite_eligible"], info
    assert info["probe_points"] == 65536 and info["probe_codes"] == 4
    assert 0.0 < info["lite_probe_ratio"] <= 0.5 and 0.0 < info["lite_probe_max_err"] <= 1e-3, info
    print("\nbench decoder probe:", info)


def test_high_error_decoder_routed_to_the_exact_path(monkeypatch):
    """A deliberately high-error decoder (hidden-weight gain 5, against the bench decoder's
    2.45: fp16 activations ~150x larger) fails the load-time qualification; every batch on it
    runs the exact HIP path — the DSR_LITE=0 kernels, not the oracle — with results bytewise
    those of DSR_LITE=0, also for warm-start codes of unit scale per component."""
    from deep_sdf.workspace import decoder_from_state

    dec = decoder_from_state(S.fit_last_layer_to_sphere(S.make_decoder_state(1234, hidden_gain=5.0)),
                             S.DEFAULT_SPECS)
    info = dec.info
    assert not info["lite_eligible"] and info["lite_probe_max_err"] > 1e-3, info
    print("\ngain-5 decoder probe:", info)
    opt = _opt(dec, S.KITTI_OPTIM, iters=2)
    rng = np.random.default_rng(5)
    objs = []
    for i, scale in enumerate((0.0, 1.0)):
        o = S.kitti_object(i)
        objs.append((o.t_cam_obj, o.pts, o.rays, o.depth, (scale * rng.standard_normal(64)).astype(np.float32)))
    monkeypatch.delenv("DSR_LITE", raising=False)
    outs, st = batch_stats(opt, objs)
    assert st.lite == 0 and st.lite_eligible == 0 and st.refine_points == 0 and st.fwd_points > 0
    monkeypatch.setenv("DSR_LITE", "0")
    ref, st0 = batch_stats(opt, objs)
    assert bytes(outs) == bytes(ref)
    assert st.fwd_points == st0.fwd_points


def _violating_batch(opt, objs, monkeypatch):
    """A resident batch whose every object sees audit violations (DSR_LITE_PERTURB)."""
    from reconstruct import _libdsr as L

    monkeypatch.setenv("DSR_LITE", "1")
    monkeypatch.setenv("DSR_TEST_HOOKS", "1")
    monkeypatch.setenv("DSR_LITE_PERTURB", "0.015")
    keep = []
    ins = (L.ObjectIn * len(objs))()
    for i, ob in enumerate(objs):
        ins[i] = opt._object_in(*ob[:4], ob[4], keep, True)
    ctx = opt._ctx
    h = C.c_void_p()
    ctx.check(ctx.lib.dsr_batch_create(ctx.handle, opt.decoder.handle, C.byref(opt.params), len(objs), ins,
                                       C.byref(h)), "create")
    return h, keep


def test_graph_replays_redo_the_spare_iteration(gpu_decoder, monkeypatch):
    """DSR_GRAPH=1 re-runs replay the captured regular iterations; a run whose audit discards
    an iteration still gets its spare iteration on every replay (the spare flag
    was left set by the previous run, so replays 3.. skipped it and reported is_good=0)."""
    from reconstruct import _libdsr as L

    f = golden("f4_traj_kitti0.npz")
    opt = _opt(gpu_decoder, S.KITTI_OPTIM, iters=2)
    objs = [(f["it_t_obj_cam"][e], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][e]) for e in (0, 4)]
    monkeypatch.setenv("DSR_GRAPH", "1")
    h, keep = _violating_batch(opt, objs, monkeypatch)
    ctx = opt._ctx
    runs = []
    try:
        for _ in range(3):
            outs = (L.ObjectOut * len(objs))()
            ctx.check(ctx.lib.dsr_batch_run(h), "run")
            ctx.check(ctx.lib.dsr_batch_download(h, outs), "download")
            st = L.Stats()
            ctx.check(ctx.lib.dsr_batch_stats(h, C.byref(st)), "stats")
            assert st.lite_redo_objects == len(objs)
            for o in outs:
                assert o.is_good == 1 and o.iters_done == 2, (o.is_good, o.iters_done, o.fail_reason)
            runs.append(bytes(outs))
    finally:
        ctx.lib.dsr_batch_destroy(h)
    assert runs[0] == runs[1] == runs[2]


def test_audit_setting_is_fixed_at_batch_creation(gpu_decoder, monkeypatch):
    """A batch created with DSR_LITE_AUDIT=0 has no spare iteration; turning the variable on
    before a run must not switch the audit on for that batch (it did, a violation
    then discarded an iteration with no spare to redo it and the object came back failed)."""
    from reconstruct import _libdsr as L

    f = golden("f4_traj_kitti0.npz")
    opt = _opt(gpu_decoder, S.KITTI_OPTIM, iters=1)
    objs = [(f["it_t_obj_cam"][0], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][0])]
    monkeypatch.setenv("DSR_LITE_AUDIT", "0")
    h, keep = _violating_batch(opt, objs, monkeypatch)
    ctx = opt._ctx
    try:
        monkeypatch.setenv("DSR_LITE_AUDIT", "1")
        outs = (L.ObjectOut * 1)()
        ctx.check(ctx.lib.dsr_batch_run(h), "run")
        ctx.check(ctx.lib.dsr_batch_download(h, outs), "download")
        st = L.Stats()
        ctx.check(ctx.lib.dsr_batch_stats(h, C.byref(st)), "stats")
    finally:
        ctx.lib.dsr_batch_destroy(h)
    assert st.lite_audit_violations == 0 and st.audit_points == 0
    assert outs[0].is_good == 1 and outs[0].iters_done == 1


def test_query_never_waits_for_the_redo(gpu_decoder, monkeypatch):
    """dsr_batch_query enqueues a pending audit redo and reports the batch as still in flight
    instead of waiting for it (the async keyframe API's overlap); polling to completion gives
    the synchronous result.  A batch captured as a graph but never run cannot be queried."""
    import time

    from reconstruct import _libdsr as L

    f = golden("f4_traj_kitti0.npz")
    opt = _opt(gpu_decoder, S.KITTI_OPTIM, iters=1)
    objs = [(f["it_t_obj_cam"][e], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][e]) for e in (0, 4)]
    h, keep = _violating_batch(opt, objs, monkeypatch)
    ctx = opt._ctx
    lib = ctx.lib
    try:
        ctx.check(lib.dsr_batch_run(h), "run")
        seen, slow = [], 0.0
        for _ in range(100000):
            t0 = time.perf_counter()
            rc = lib.dsr_batch_query(h)
            slow = max(slow, time.perf_counter() - t0)
            assert rc >= 0
            seen.append(rc)
            if rc == 1:
                break
        assert seen[-1] == 1
        polled = (L.ObjectOut * 2)()
        ctx.check(lib.dsr_batch_download(h, polled), "download")
        ctx.check(lib.dsr_batch_run(h), "run")
        synced = (L.ObjectOut * 2)()
        ctx.check(lib.dsr_batch_download(h, synced), "download")
        assert bytes(polled) == bytes(synced)
        assert all(o.is_good == 1 and o.iters_done == 1 for o in polled)
        print(f"\nlongest query {slow * 1e3:.3f} ms over {len(seen)} polls")
    finally:
        lib.dsr_batch_destroy(h)
    monkeypatch.setenv("DSR_GRAPH", "1")
    h, keep = _violating_batch(opt, objs, monkeypatch)
    try:
        ctx.check(lib.dsr_batch_graph(h), "graph")
        assert lib.dsr_batch_query(h) < 0          # captured, never run
    finally:
        lib.dsr_batch_destroy(h)



def test_stats_report_the_kernels_the_run_dispatched(gpu_decoder, monkeypatch):
    """dsr_stats' kernel fields (ABI 10/11) are the kernels the last run
    dispatched, resolved as it was enqueued — an unknown DSR_LITE_VARIANT runs (and reports) the
    shipped 1496, and changing the environment between run and stats changes nothing reported."""
    from reconstruct import _libdsr as L

    opt = _opt(gpu_decoder, S.KITTI_OPTIM, "KITTI", iters=2)
    objs = [(o.t_cam_obj, o.pts, o.rays, o.depth, None) for o in (S.kitti_object(i) for i in range(2))]
    monkeypatch.setenv("DSR_TEST_HOOKS", "1")
    monkeypatch.setenv("DSR_LITE_VARIANT", "16")       # not a kernel of the shipped build
    keep = []
    ins = (L.ObjectIn * 2)()
    for i, ob in enumerate(objs):
        ins[i] = opt._object_in(*ob[:4], None, keep)
    ctx = opt._ctx
    h = C.c_void_p()
    ctx.check(ctx.lib.dsr_batch_create(ctx.handle, opt.decoder.handle, C.byref(opt.params), 2, ins,
                                       C.byref(h)), "create")
    try:
        ctx.check(ctx.lib.dsr_batch_run(h), "run")
        ctx.check(ctx.lib.dsr_batch_sync(h), "sync")
        monkeypatch.setenv("DSR_FWD_VARIANT", "0")     # after the run: must not be reported
        monkeypatch.setenv("DSR_JAC_VARIANT", "0")
        monkeypatch.setenv("DSR_SPLIT_RING", "3")
        st = L.Stats()
        ctx.check(ctx.lib.dsr_batch_stats(h, C.byref(st)), "stats")
    finally:
        ctx.lib.dsr_batch_destroy(h)
    assert (st.lite_variant, st.fwd_variant, st.jac_variant, st.split_ring) == (1496, 12, 12, 2)
    assert st.n_groups == 2 and st.prescan == 0
