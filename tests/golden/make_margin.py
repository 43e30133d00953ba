"""Margin-screened trajectory fixtures (F8): the north-star output contract.

Build-container only (imports the REFERENCE through ``refshim``).  Usage::

    python tests/golden/make_margin.py [--quick]    # writes tests/golden/f8_*.npz

Why screening: ``Optimizer.reconstruct_object`` (reference optimizer.py:90-205) is
a piecewise-smooth map of its inputs.  Its pieces are cut by four discontinuous
masks (SURVEY.md §7 "Hard parts"):

* ``|x_obj| < 1``     — a ray sample enters the decoded set (loss.py:79);
* ``|sdf| < th``      — a sample becomes a render point (loss.py:101-102);
* ``de_do > 1e-2``    — a render point keeps its gradient (loss.py:135);
* ``res_rot < 1e-7``  — the upright prior switches on (loss.py:185-186; with
  KITTI's k4 = 1e7 this is a large jump in H).

Any implementation whose fp32 rounding differs from the reference's (another
thread count of the reference itself, the build's MFMA decoder) lands on the
other side of a threshold whenever the reference's own trajectory passes closer
to it than that rounding, and from then on the two trajectories are different
GN runs.  The Huber switches (loss_utils.py:246-259) and the +-0.30 residual
clamp (loss.py:147-148) are continuous in the residual fed to b, so they only
record a margin here.

For each candidate object the reference runs at ``torch.set_num_threads(1)``;
every iteration's state (pose, code, sample depths) and the decoder values it
computed are recorded, and the distance of every RELEVANT sample to each
threshold is measured:

* band: ``| |sdf| - th |`` over in-ball samples whose transmittance in front of
  them is non-zero (behind a full sample, loss.py:111 multiplies by exact zero);
* de_do: ``|de_do / 1e-2 - 1|`` over the render candidates (``|sdf| < th``);
* ball: ``| |x| - 1 |`` over samples with ``sdf < th`` and non-zero transmittance
  in front (an empty sample flipping in or out of the ball changes nothing but
  N_valid); ``ball_all`` over every sample (exact N_valid);
* rot: distance of the fp32 ``R_co[1,1]`` from the rounding boundary that
  decides ``res_rot < 1e-7``, in units of 2^-24 (an fp32 ulp below 1).

A candidate is kept only if every iteration's margins clear ``ACCEPT`` —
about 10x the GPU-vs-reference SDF error (~1e-6, tests/test_gpu_parity.py).

There is a fifth discontinuity that cannot be screened away: every hidden ReLU of
every Jacobian point (the N surface points and K render points go through
autograd, loss_utils.py:82-113).  The SDF is continuous across a kink but its
gradient is not; a pre-activation within fp32 rounding of zero flips its mask in
one implementation and not in another, and that point's Jacobian row jumps by a
few percent.  With ~4,000 hidden units per point, any two fp32 implementations
(the reference at 1 vs 8 threads included) disagree on a few points per
iteration: H differs by ~1e-4 relative, the step by ~1e-4 x cond(H).  Whether
that stays small over the whole trajectory is a property of the input: for
some objects the GN map contracts such differences, for others (nearly
unobservable yaw of a round shape, KITTI's stiff k4 = 1e7 prior with its fp32
res_rot staircase) it amplifies them to 1e-2 within a few iterations.  So the
second screen is the reference's own sensitivity: the trajectory is re-run from
the initial pose perturbed at the 1e-7 relative level (one fp32 ulp) ``ENSEMBLE``
times; the candidate is kept only if every member keeps the same K at every
iteration and lands within
``SPREAD_MAX`` (the contract itself) of the 1-thread result.  On inputs
that pass both screens the build must reproduce the reference's final
``t_cam_obj``, ``code`` and ``loss`` (optimizer.py:202-205) to the north star's
1e-3 / 1e-4.  The third screen (round 6, ``--conditioning``) is the GN step's own
conditioning at the fp32 level (tools/f8_conditioning.py): from every recorded state,
perturbed by as much as the fp32 oracle's own state is off there, the fp64 oracle's next
state must stay within the contract — otherwise no implementation that rounds
differently from the reference can be held to the fixture's end point.  Candidates use
fewer rays than the bench object (fewer samples near a threshold); the measured margins and spreads of rejected candidates are stored
too (``f8_screen.npz``), including full-size 2048-point KITTI objects, to show
what does not qualify and why.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, HERE)

import synthetic as S  # noqa: E402
import refshim  # noqa: E402
import make_golden as MG  # noqa: E402

#: acceptance: every iteration, every relevant sample at least this far from a threshold
ACCEPT = {"band": 1e-5, "dedo": 1e-3, "ball": 1e-5, "rot_ulps": 4.0}
#: second screen: the reference's own 8-thread / 1-ulp-perturbed runs vs its 1-thread run
SPREAD_MAX = {"pose": 1e-3, "code": 1e-3, "loss": 1e-4}
#: members of that ensemble: the initial pose perturbed at the 1e-7 level, 1 thread each
#: (torch's multi-threaded CPU reductions are not run-to-run deterministic on a loaded host,
#: which would make the screen itself irreproducible)
ENSEMBLE = 8
HALF_ULP_BOUNDARY = 1.5 * 2.0 ** -24      # fp32 res_rot < 1e-7  <=>  1 - R_co[1,1]... rounds below this


def reduce_rays(ob, n_fg, n_bg):
    """The object with only its first ``n_fg`` foreground and ``n_bg`` background rays."""
    n_all_fg = ob.depth.shape[0]
    rays = np.concatenate([ob.rays[:n_fg], ob.rays[n_all_fg:n_all_fg + n_bg]]).astype(np.float32)
    return S.SyntheticObject(ob.t_cam_obj, ob.pts, rays, ob.depth[:n_fg].copy(), ob.t_true)


def tilted(ob, seed):
    """``ob`` with its initial pose tilted by 2-5 mrad about the camera x axis: an exactly
    upright start puts res_rot (loss.py:181) within 1.5 fp32 ulps of its 1e-7 switch,
    a real detection never is."""
    a = np.random.default_rng(seed + 7).uniform(2e-3, 5e-3)
    Rx = np.array([[1, 0, 0], [0, np.cos(a), -np.sin(a)], [0, np.sin(a), np.cos(a)]])
    T = ob.t_cam_obj.astype(np.float64).copy()
    T[:3, :3] = Rx @ T[:3, :3]
    return S.SyntheticObject(T.astype(np.float32), ob.pts, ob.rays, ob.depth, ob.t_true)


def run_recorded(ref, dec, cfg, data_type, ob):
    """run_traj plus the decoded samples and residuals of every iteration."""
    import torch

    torch.set_num_threads(1)
    opt = refshim.make_optimizer(dec, cfg, data_type)
    with MG.Recorder(ref) as rec:
        inner_decode = ref.loss.decode_sdf
        inner_robust = ref.optimizer.get_robust_res

        def decode(decoder, z, x, *a, **k):
            out = inner_decode(decoder, z, x, *a, **k)
            rec.it[-1]["query_sdf"] = out.numpy().reshape(-1).copy()
            return out

        def robust(res, b):
            key = "res_sdf" if "res_sdf" not in rec.it[-1] else "res_render"
            rec.it[-1][key] = res.numpy().reshape(-1).copy()
            return inner_robust(res, b)

        ref.loss.decode_sdf = decode
        ref.optimizer.get_robust_res = robust
        try:
            r = opt.reconstruct_object(ob.t_cam_obj.copy(), ob.pts, ob.rays, ob.depth, None)
        finally:
            ref.loss.decode_sdf = inner_decode
            ref.optimizer.get_robust_res = inner_robust
    return r, rec.it


def iteration_margins(ref, dec, it, rays, th, k4, b1, b2):
    """Margins of one recorded iteration (module docstring)."""
    import torch

    T = torch.from_numpy(it["t_obj_cam"])
    dep = torch.from_numpy(it["depths"])
    R = torch.from_numpy(rays)
    # loss.py:72-75, same fp32 ops -> the reference's sample positions and norms
    cam = R[..., None, :] * dep[:, None]
    obj = (cam[..., None, :] * T[:3, :3]).sum(-1) + T[:3, 3]
    nrm = torch.norm(obj, dim=-1).numpy().astype(np.float64)
    inball = nrm < 1.0
    out = {"n_valid": int(inball.sum())}
    sdf = np.full(nrm.shape, np.nan)
    if "query_sdf" in it:
        sdf[inball] = it["query_sdf"].astype(np.float64)
    # out-of-ball samples near the sphere: what they would decode to if they flipped in
    near = (~inball) & (np.abs(nrm - 1.0) < 2e-3)
    if near.any():
        with torch.no_grad():
            zq = torch.from_numpy(it["z"])
            xq = obj[torch.from_numpy(near)]
            nq = xq.shape[0]
            if nq == 1:                      # decode_sdf squeezes a 1-row chunk to 0-d
                xq = torch.cat([xq, xq])
            sdf_near = ref.loss_utils.decode_sdf(dec, zq, xq).numpy().reshape(-1)[:nq].astype(np.float64)
    occ = np.where(inball, 0.5 - np.clip(np.nan_to_num(sdf, nan=1.0), -th, th) / (2 * th), 0.0)
    keep = 1.0 - occ
    acc = np.cumprod(keep, axis=1)                                   # A_l = prod_{m<=l}
    prefix = np.concatenate([np.ones((acc.shape[0], 1)), acc[:, :-1]], axis=1)
    live = prefix > 0.0
    rel_in = inball & live
    band_d = np.abs(np.abs(sdf) - th)
    out["band"] = float(band_d[rel_in].min()) if rel_in.any() else np.inf
    cand = inball & (np.abs(sdf) < th)
    if cand.any():
        tail = np.cumsum(acc[:, ::-1], axis=1)[:, ::-1]              # sum_{l>=j} A_l
        with np.errstate(divide="ignore", invalid="ignore"):
            dedo = tail / (1.0 - occ)
        d = dedo[cand]
        out["dedo"] = float(np.abs(d / 1e-2 - 1.0).min())
        out["k_fp64"] = int((d > 1e-2).sum())
    else:
        out["dedo"] = np.inf
        out["k_fp64"] = 0
    ball_rel = rel_in & (sdf < th)
    cands = [np.abs(nrm[ball_rel] - 1.0)]
    if near.any():
        nidx = np.argwhere(near)
        nr = np.abs(nrm[near] - 1.0)
        nl = live[near] & (sdf_near < th)
        cands.append(nr[nl])
        del nidx
    cc = np.concatenate(cands)
    out["ball"] = float(cc.min()) if cc.size else np.inf
    out["ball_all"] = float(np.abs(nrm - 1.0).min())
    if "res_render" in it and it["res_render"].size:
        rr = np.abs(it["res_render"].astype(np.float64))
        unclamped = rr[rr != np.float64(np.float32(0.30))]      # clamped values sit exactly on it
        out["clamp"] = float(np.abs(unclamped - 0.30).min()) if unclamped.size else np.inf
        out["huber_render"] = float(np.abs(rr - b1).min())
    if "res_sdf" in it and it["res_sdf"].size:
        out["huber_sdf"] = float(np.abs(np.abs(it["res_sdf"].astype(np.float64)) - b2).min())
    if k4 != 0.0:
        # loss.py:175-186 in fp32: R_co[1,1] decides res_rot = 1 - (-R_co[1,1]) < 1e-7
        t_co = np.linalg.inv(it["t_obj_cam"].astype(np.float64))
        rco = t_co[:3, :3] / np.cbrt(np.linalg.det(t_co[:3, :3]))
        res64 = 1.0 + rco[1, 1]
        out["res_rot"] = float(res64)
        out["rot_ulps"] = float(abs(res64 - HALF_ULP_BOUNDARY) / 2.0 ** -24)
    else:
        out["rot_ulps"] = np.inf
    return out


def contract_errors(r, base):
    """(pose, code, loss) relative differences of result ``r`` vs ``base`` (reference
    results), as tests/test_gpu_contract.py measures them."""
    if not (r.is_good and base.is_good):
        return np.inf, np.inf, np.inf
    T, Tb = np.asarray(r.t_cam_obj, np.float64), np.asarray(base.t_cam_obj, np.float64)
    e_p = max(np.abs(T[:3, :3] - Tb[:3, :3]).max() / np.abs(Tb[:3, :3]).max(),
              np.abs(T[:3, 3] - Tb[:3, 3]).max() / np.abs(Tb[:3, 3]).max())
    zb = np.asarray(base.code, np.float64)
    e_z = np.abs(np.asarray(r.code, np.float64) - zb).max() / np.abs(zb).max()
    e_l = abs(float(r.loss) - float(base.loss)) / abs(float(base.loss))
    return float(e_p), float(e_z), float(e_l)


def ensemble_spread(ref, dec, cfg, data_type, ob, base, base_k=None, members=None):
    """Max (pose, code, loss) difference of the reference's perturbed runs from ``base``
    (inf if a member's render-point count K differs from ``base_k`` at any iteration).
    ``members`` (a list) receives each member's final (t_cam_obj, code, loss)."""
    prng = np.random.default_rng(77)
    spread = np.zeros(3)
    for k in range(ENSEMBLE):
        T = ob.t_cam_obj.astype(np.float64)
        T[:3, :] *= 1.0 + 1e-7 * prng.standard_normal((3, 4))
        ob2 = S.SyntheticObject(T.astype(np.float32), ob.pts, ob.rays, ob.depth, ob.t_true)
        r2, its2 = MG.run_traj(ref, dec, cfg, data_type, ob2, threads=1)
        spread = np.maximum(spread, contract_errors(r2, base))
        if members is not None:
            members.append((np.asarray(r2.t_cam_obj if r2.is_good else np.full((4, 4), np.nan), np.float32),
                            np.asarray(r2.code if r2.is_good else np.full(64, np.nan), np.float32),
                            float(r2.loss)))
        if base_k is not None and [i.get("k", -1) for i in its2] != base_k:
            spread[:] = np.inf
        if (spread > [SPREAD_MAX["pose"], SPREAD_MAX["code"], SPREAD_MAX["loss"]]).any():
            break                       # already rejected
    import torch

    torch.set_num_threads(1)
    return spread


_COND = None


def conditioning_of(out):
    """tools/f8_conditioning.py's record for a packed candidate (``out``: the fixture arrays)"""
    global _COND
    if _COND is None:
        sys.path.insert(0, os.path.join(REPO, "tools"))
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import f8_conditioning as FC

        _COND = (FC, FC.decoders())
    FC, (d64, d32) = _COND
    return FC.conditioning(out, d64, d32)


def screen(ref, dec, name, cfg, data_type, ob):
    jo = cfg["joint_optim"]
    t0 = time.time()
    r, its = run_recorded(ref, dec, cfg, data_type, ob)
    ms = [iteration_margins(ref, dec, it, ob.rays, cfg["cut_off_threshold"], jo["k4"], jo["b1"], jo["b2"])
          for it in its if "depths" in it]
    keys = ("band", "dedo", "ball", "ball_all", "rot_ulps", "clamp", "huber_render", "huber_sdf")
    mins = {k: float(min(m.get(k, np.inf) for m in ms)) if ms else np.nan for k in keys}
    ok = bool(r.is_good) and all(mins[k] >= v for k, v in ACCEPT.items())
    # sanity: the fp64 re-evaluation reproduces the reference's own N_valid / K
    nv_ok = all(m["n_valid"] == it.get("n_valid", -1) for m, it in zip(ms, its))
    k_ok = all(m["k_fp64"] == it.get("k", -1) for m, it in zip(ms, its))
    spread = np.full(3, np.nan)
    members = []
    if ok and nv_ok and k_ok:
        spread = ensemble_spread(ref, dec, cfg, data_type, ob, r, [i.get("k", -1) for i in its], members)
        ok = bool((spread <= [SPREAD_MAX["pose"], SPREAD_MAX["code"], SPREAD_MAX["loss"]]).all())
    mins["spread_pose"], mins["spread_code"], mins["spread_loss"] = (float(x) for x in spread)
    mins["members"] = members
    print(f"  {name}: good={bool(r.is_good)} ok={ok} nv={nv_ok} k={k_ok} "
          + " ".join(f"{k}={mins[k]:.2e}" for k in keys)
          + " spread=" + "/".join(f"{x:.1e}" for x in spread) + f" ({time.time() - t0:.1f}s)", flush=True)
    return r, its, ms, mins, ok, nv_ok and k_ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="fewer candidates (smoke)")
    ap.add_argument("--seeds", default="", help="only these seeds, e.g. 5220,5182,6045")
    ap.add_argument("--no-full", action="store_true", help="skip the full-size KITTI objects")
    ap.add_argument("--family", default="", help="only these families, e.g. redwood3it,kitti3it")
    ap.add_argument("--screen-file", default="f8_screen.npz")
    ap.add_argument("--seed-base", type=int, default=-1, help="first seed (default 5000 / 6000)")
    ap.add_argument("--tries", type=int, default=-1, help="candidates per family (default: the family's)")
    ap.add_argument("--conditioning", action="store_true",
                    help="also require a well-conditioned GN step at every iteration (round 6)")
    args = ap.parse_args()
    only = {int(x) for x in args.seeds.split(",") if x.strip()}
    import torch

    torch.set_num_threads(1)
    ref = refshim.load()
    dec = refshim.build_decoder(S.make_decoder(MG.DECODER_SEED), S.DEFAULT_SPECS)
    meta = {"torch": np.array(torch.__version__), "numpy": np.array(np.__version__),
            "accept": np.array([ACCEPT[k] for k in ("band", "dedo", "ball", "rot_ulps")]),
            "accept_keys": np.array(["band", "dedo", "ball", "rot_ulps"])}
    def iters(cfg, n):
        return dict(cfg, joint_optim=dict(cfg["joint_optim"], num_iterations=n))

    redwood = lambda s: S.make_object(s, n_pts=512, scale=1.0, tz=3.0, upright=False)  # noqa: E731
    kitti = lambda s: tilted(S.make_object(s, n_pts=2048, scale=2.0, tz=15.0, upright=True), s)  # noqa
    kitti512 = lambda s: tilted(S.make_object(s, n_pts=512, scale=2.0, tz=15.0, upright=True), s)  # noqa
    redwood2048 = lambda s: S.make_object(s, n_pts=2048, scale=1.0, tz=3.0, upright=False)  # noqa: E731
    families = [
        # (tag, optim, data_type, object factory(seed), n_fg, n_bg, wanted, max tries)
        ("redwood", S.REDWOOD_OPTIM, "Redwood", redwood, 32, 8, 2, 400),
        ("kitti", S.KITTI_OPTIM, "KITTI", kitti, 32, 8, 2, 400),
        # the same parameter sets with 3 GN iterations (joint_optim.num_iterations is a
        # config value of the reference): fewer mask crossings to amplify, so some inputs
        # are reproducible to the contract where the full iteration counts found none
        ("redwood3it", iters(S.REDWOOD_OPTIM, 3), "Redwood", redwood, 32, 8, 2, 200),
        ("kitti3it", iters(S.KITTI_OPTIM, 3), "KITTI", kitti, 32, 8, 2, 200),
        # round 3: KITTI parameters (upright prior k4 = 1e7 active: the tilted start keeps
        # res_rot > 1e-7, its fp32 rounding boundary recorded as margin_rot_ulps) with 2 GN
        # iterations — 3 found none whose 8-member ensemble stayed within the contract (the
        # code spreads 1e-3..1e-2 through the Jacobian points' ReLU kinks, amplified by the
        # weakly regularised code block of H: k3 = 0.25); ~2% of 2-iteration inputs qualify
        ("kitti2it", iters(S.KITTI_OPTIM, 2), "KITTI", kitti, 32, 8, 3, 200),
        ("kitti2it_r64", iters(S.KITTI_OPTIM, 2), "KITTI", kitti, 64, 8, 2, 200),
        ("kitti2it_p512", iters(S.KITTI_OPTIM, 2), "KITTI", kitti512, 32, 8, 2, 200),
        # round 6: the Redwood parameter set at its own 5 iterations
        # (config_redwood_01053.json:26), screened with --conditioning.  Each hidden-ReLU kink
        # flip of a Jacobian point moves H by ~1/N of that point's share (the sdf term is a mean
        # over N surface points, the render term over K), so more surface points and fewer rays
        # make each flip smaller: 2048 points, 16 + 4 rays
        ("redwood5_p2048_r16", S.REDWOOD_OPTIM, "Redwood", redwood2048, 16, 4, 2, 400),
        ("redwood5_p2048", S.REDWOOD_OPTIM, "Redwood", redwood2048, 32, 8, 2, 400),
        ("redwood5_r16", S.REDWOOD_OPTIM, "Redwood", redwood, 16, 4, 2, 400),
    ]
    if args.family:
        families = [f for f in families if f[0] in args.family.split(",")]
    if args.quick:
        families = [(f[0], f[1], f[2], f[3], f[4], f[5], 1, 3) for f in families]
    screened = []
    for tag, cfg, dtp, fac, n_fg, n_bg, want, tries in families:
        got = 0
        if args.tries > 0:
            tries = args.tries
        for k in range(tries):
            base = args.seed_base if args.seed_base >= 0 else (5000 if tag.startswith("redwood") else 6000)
            seed = base + k
            if only and seed not in only:
                continue
            ob = reduce_rays(fac(seed), n_fg, n_bg)
            name = f"{tag}_s{seed}"
            r, its, ms, mins, ok, consistent = screen(ref, dec, name, cfg, dtp, ob)
            screened.append((name, ok, consistent, mins))
            if not (ok and consistent):
                continue
            out = MG.pack_traj(r, its)
            if args.conditioning:
                out_c = dict(out, obj_t_cam_obj=ob.t_cam_obj, obj_pts=ob.pts, obj_rays=ob.rays, obj_depth=ob.depth,
                             data_type=np.array(dtp), num_iterations=np.array(cfg["joint_optim"]["num_iterations"]))
                c = conditioning_of(out_c)
                mins["cond_worst"] = max(c["worst_next_state_deviation"], default=0.0)
                print(f"    conditioning: worst next-state deviation "
                      f"{' '.join(f'{w:.1e}' for w in c['worst_next_state_deviation'])}"
                      f" -> {'ok' if c['well_conditioned'] else 'ILL-CONDITIONED'}", flush=True)
                if not c["well_conditioned"]:
                    screened[-1] = (name, False, consistent, mins)
                    continue
            out.update({"obj_t_cam_obj": ob.t_cam_obj, "obj_pts": ob.pts, "obj_rays": ob.rays,
                        "obj_depth": ob.depth, "seed": np.array(seed), "data_type": np.array(dtp),
                        "n_fg": np.array(n_fg), "n_bg": np.array(n_bg),
                        "num_iterations": np.array(cfg["joint_optim"]["num_iterations"])})
            for key in ("band", "dedo", "ball", "ball_all", "rot_ulps", "clamp", "huber_render",
                        "huber_sdf"):
                out["margin_" + key] = np.array([m.get(key, np.inf) for m in ms])
            out["ref_spread"] = np.array([mins["spread_pose"], mins["spread_code"], mins["spread_loss"]])
            out["ens_t_cam_obj"] = np.stack([m[0] for m in mins["members"]])
            out["ens_code"] = np.stack([m[1] for m in mins["members"]])
            out["ens_loss"] = np.array([m[2] for m in mins["members"]])
            np.savez_compressed(os.path.join(HERE, f"f8_margin_{name}.npz"), **out, **meta)
            got += 1
            if got >= want:
                break
    # full-size bench objects (2048 pts x 2248 rays): margins measured, expected not to qualify
    if not args.quick and not args.no_full:
        for i in range(2):
            ob = S.kitti_object(i)
            r, its, ms, mins, ok, consistent = screen(ref, dec, f"kitti_full{i}", S.KITTI_OPTIM, "KITTI", ob)
            if not ok:                   # record the full-size reference's own spread as well
                sp = ensemble_spread(ref, dec, S.KITTI_OPTIM, "KITTI", ob, r)
                mins["spread_pose"], mins["spread_code"], mins["spread_loss"] = (float(x) for x in sp)
            screened.append((f"kitti_full{i}", ok, consistent, mins))
    keys = ("band", "dedo", "ball", "ball_all", "rot_ulps", "clamp", "huber_render", "huber_sdf",
            "spread_pose", "spread_code", "spread_loss") + (("cond_worst",) if args.conditioning else ())
    np.savez_compressed(os.path.join(HERE, args.screen_file),
                        names=np.array([s[0] for s in screened]), ok=np.array([s[1] for s in screened]),
                        consistent=np.array([s[2] for s in screened]),
                        margins=np.array([[s[3].get(k, np.nan) for k in keys] for s in screened]),
                        margin_keys=np.array(keys), **meta)


if __name__ == "__main__":
    main()
