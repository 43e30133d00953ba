"""Every lite classification checked by the real kernel (GPU): the lite pass's safety measured
on full GN trajectories instead of emulated (tools/lite_error_survey.py is the numpy emulation).

With DSR_LITE_AUDIT_LOG2=0 the audit's hashed share is 2^0: the exact split-fp16 pass re-decodes
every sample the lite pass decoded up to its ray's first certainly-full one (the ones behind it sit
at transmittance 0 and cannot affect an output), records |lite - exact| (dsr_stats.lite_max_err) and compares
the two classes (full <= -th | band | empty >= th) outside the band (lite_audit_violations; a
violation discards that object's iteration and redoes it exactly).  Run over decoders of three
hidden-weight gains, warm-start codes of three scales and 64 KITTI objects x 10 iterations, at
  A: the shipped margins (first iteration th, then max(0.002, 4 x observed error)),
  B: a fixed 0.002 margin (the floor alone: DSR_LITE_SAFETY=0),
  C: a fixed 0.001 margin (half the floor: what the margin has in hand).

Usage (GPU box): python tools/lite_audit_all.py [n_decoders]   -> one line per run + totals
"""
from __future__ import annotations

import ctypes as C
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)

import synthetic as S  # noqa: E402

SETTINGS = {"A": {}, "B": {"DSR_LITE_SAFETY": "0"},
            "C": {"DSR_LITE_SAFETY": "0", "DSR_LITE_FLOOR": "0.001"}}


def main():
    from deep_sdf.workspace import decoder_from_state
    from reconstruct import _libdsr as L
    from reconstruct.optimizer import Optimizer
    from reconstruct.parallel import ResidentShard
    from reconstruct.utils import ForceKeyErrorDict

    n_dec = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    n_obj = int(os.environ.get("AUDIT_ALL_OBJECTS", "64"))
    os.environ["DSR_LITE_AUDIT_LOG2"] = "0"            # read at batch creation
    rng = np.random.default_rng(11)
    tot = {k: [0, 0, 0, 0.0, 0] for k in SETTINGS}    # audited, decoded, violations, max err, redo objects
    print("setting | decoder (seed, gain) | code scale | decoded | audited | band (refined) | violations | redo objects | "
          "max |lite - exact| | min margin | good", flush=True)
    t0 = time.time()
    for k in range(n_dec):
        seed, gain = 1234 + 17 * k, (2.45, 2.0, 3.2)[k % 3]
        state = S.fit_last_layer_to_sphere(S.make_decoder_state(seed, hidden_gain=gain))
        dec = decoder_from_state(state, S.DEFAULT_SPECS, device=0)
        opt = Optimizer(dec, ForceKeyErrorDict(data_type="KITTI", optimizer=S.KITTI_OPTIM))
        lib, ctx = dec.ctx.lib, dec.ctx
        for cs in (0.0, 0.3, 1.0):
            objs = []
            for i in range(n_obj):
                o = S.kitti_object(i, base_seed=7000 + 100 * k)
                z = None if cs == 0.0 else (cs * rng.standard_normal(64)).astype(np.float32)
                objs.append((o.t_cam_obj, o.pts, o.rays, o.depth, z))
            for name, env in SETTINGS.items():
                saved = {v: os.environ.get(v) for v in env}
                os.environ.update(env)
                try:
                    sh = ResidentShard(opt, objs)
                finally:
                    for v, old in saved.items():
                        if old is None:
                            os.environ.pop(v, None)
                        else:
                            os.environ[v] = old
                try:
                    res = sh.run()
                    st = L.Stats()
                    ctx.check(lib.dsr_batch_stats(sh.handle, C.byref(st)), "stats")
                finally:
                    sh.close()
                good = sum(int(r["is_good"]) for r in res)
                t = tot[name]
                t[0] += st.audit_points
                t[1] += st.fwd_points
                t[2] += st.lite_audit_violations
                t[3] = max(t[3], st.lite_max_err)
                t[4] += st.lite_redo_objects
                print(f"{name} | ({seed}, {gain}) | {cs} | {st.fwd_points} | {st.audit_points} | {st.refine_points - st.audit_points} | "
                      f"{st.lite_audit_violations} | {st.lite_redo_objects} | {st.lite_max_err:.3e} | "
                      f"{st.lite_min_margin:.4f} | {good}/{n_obj}", flush=True)
    print(f"totals ({time.time() - t0:.0f} s):")
    for name, (aud, decd, vio, err, redo) in tot.items():
        print(f"  {name}: {decd} lite-decoded sample-iterations, {aud} audited ({aud / max(1, decd):.3f}), "
              f"{vio} class violations, {redo} objects redone, max |lite - exact| {err:.3e}", flush=True)


if __name__ == "__main__":
    main()
