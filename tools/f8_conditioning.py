"""Conditioning of the margin-screened fixtures (golden F8) at the fp32 level (CPU, fp64 oracle).

The strict contract test (tests/test_gpu_contract.py: test_final_state_matches_reference) holds
a GPU trajectory to 1e-3 of the reference's pose / code at every iteration.  The fixtures were
screened for mask margins at the reference's states and for an 8-member ulp ensemble of the
reference staying together — not for how far ONE GN step moves when its starting state is off by
what fp32 rounding leaves after a few steps.  Here, at every recorded state but the last, the
state is perturbed by as much as a correct fp32 implementation's own state is off there — the fp32
oracle's trajectory from the same start, its pose deviation from the reference's at that
iteration (at least 1e-7) — in random directions (fixed seed), the fp64 oracle takes the step,
and the next state's code / pose deviation from the reference's next state is recorded.  The perturbation is a Sim(3) one, T' = exp_sim3(xi) T (the update's own form,
optimizer.py:192), xi a random 7-vector of max-norm `mag` (rotation in radians, translation,
log-scale) — not an entry-wise one, which would break the rotation and wake the k4 = 1e7 upright
prior.  A fixture whose worst deviation exceeds the contract (1e-3) cannot be held to it by an fp32
implementation that rounds differently from the reference; it is reported, with the numbers, as
ill-conditioned, and the strict test holds it to the oracle's step from the GPU's own states
instead (tests/test_gpu_contract.py).

usage: python tools/f8_conditioning.py  ->  tests/golden/f8_conditioning.json
"""
from __future__ import annotations

import glob
import json
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
import synthetic as S  # noqa: E402
from deep_sdf.workspace import fold_state  # noqa: E402
from oracle import dsr_oracle as O  # noqa: E402
from test_gpu_contract import optim_of  # noqa: E402

N_DIR, CONTRACT, FLOOR = 6, 1e-3, 1e-7


def conditioning(path, d64, d32):
    """{perturbation, worst_next_state_deviation, well_conditioned} of one F8 fixture (a path, or
    the fixture's arrays as a mapping: tests/golden/make_margin.py screens candidates with it)"""
    f = np.load(path, allow_pickle=False) if isinstance(path, str) else path
    optim, _ = optim_of(_Files(f))
    P = O.OptimParams.from_cfg(optim)
    n_fg = f["obj_depth"].shape[0]
    dobs = np.concatenate([f["obj_depth"], np.zeros(f["obj_rays"].shape[0] - n_fg)])
    pts, rays = f["obj_pts"].astype(np.float64), f["obj_rays"].astype(np.float64)
    rng = np.random.default_rng(0)
    # the fp32 oracle's own trajectory: how far a correct fp32 implementation's state is off
    T, z = np.linalg.inv(np.asarray(f["obj_t_cam_obj"], np.float64)).astype(np.float32), np.zeros(64, np.float32)
    mags = []
    for e in range(int(f["n_iters_run"])):
        Tr = f["it_t_obj_cam"][e].astype(np.float64)
        mags.append(max(FLOOR, float(np.abs(T.astype(np.float64) - Tr).max() / np.abs(Tr).max())))
        _, T, z = O.gn_step(d32, P, T, z, pts.astype(np.float32), rays.astype(np.float32), dobs.astype(np.float32), n_fg)
        if T is None:
            break
    worst = []
    for e in range(int(f["n_iters_run"]) - 1):
        T0, z0 = f["it_t_obj_cam"][e].astype(np.float64), f["it_z"][e].astype(np.float64)
        Tn_r, zn_r = f["it_t_obj_cam"][e + 1].astype(np.float64), f["it_z"][e + 1].astype(np.float64)
        w = 0.0
        for _ in range(N_DIR):
            xi = rng.standard_normal(7)
            xi *= mags[e] / np.abs(xi).max()
            _, Tn, zn = O.gn_step(d64, P, O.exp_sim3(xi) @ T0, z0, pts, rays, dobs, n_fg)
            if Tn is None:
                w = float("inf")
                continue
            dp = np.abs(Tn - Tn_r).max() / np.abs(Tn_r).max()
            dz = np.abs(zn - zn_r).max() / max(np.abs(zn_r).max(), 1e-30)
            w = max(w, dp, dz)
        worst.append(w)
    return {"perturbation": mags[:len(worst)], "worst_next_state_deviation": worst,
            "well_conditioned": bool(max(worst, default=0.0) <= CONTRACT)}


class _Files(dict):
    """a mapping with NpzFile's ``.files``, as optim_of reads it"""

    def __init__(self, f):
        super().__init__({k: f[k] for k in (f.files if hasattr(f, "files") else f.keys())})
        self.files = list(self.keys())


def decoders():
    layers = fold_state(S.make_decoder(1234), S.DEFAULT_SPECS)
    return O.Decoder(layers, dtype=np.float64), O.Decoder(layers)


def main():
    d64, d32 = decoders()
    out = {"perturbation": "the fp32 oracle's own pose deviation at the iteration (>= 1e-7)", "directions": N_DIR,
           "contract": CONTRACT, "fixtures": {}}
    for path in sorted(glob.glob(os.path.join(REPO, "tests", "golden", "f8_margin_*.npz"))):
        name = os.path.basename(path)[len("f8_margin_"):-4]
        c = out["fixtures"][name] = conditioning(path, d64, d32)
        print(f"{name}: perturbation {' '.join(f'{m:.0e}' for m in c['perturbation'])} -> worst next-state "
              f"deviation {' '.join(f'{w:.1e}' for w in c['worst_next_state_deviation'])}"
              f" -> {'ok' if c['well_conditioned'] else 'ILL-CONDITIONED'}", flush=True)
    with open(os.path.join(REPO, "tests", "golden", "f8_conditioning.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
