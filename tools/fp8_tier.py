"""Would an FP8 pre-classification tier pay?  (numpy, runs on CPU.)

The lite pass decodes every ray sample the render term needs with ONE fp16
product and only has to tell empty (sdf >= th) / full (sdf <= -th) / band apart
(loss_utils.py:40-48, loss.py:98-102).  An fp8 tier on v_mfma_f32_16x16x128_f8f6f4 (2x the fp16
rate) would classify first and send only what it cannot certify to the fp16 lite pass.  This tool
emulates that tier — e4m3 (OCP e4m3fn: 3 mantissa bits, max 448) weights per layer (per-row power-
of-two scale, as the split packs scale per layer) and activations per 128-point tile and layer,
exact products, fp32 accumulation from the bias, fp32 lin0 and lin8 — on the samples of every
recorded state of the golden F4 KITTI trajectories (the metric objects, 10 GN iterations), and
counts the share of the lite-decoded samples (in-ball, up to each ray's first certainly-full
sample: what early ray termination leaves) it would certify with the lite pass's own rule: margin
= max(0.002, 4 x the largest |fp8 - exact| the object's band samples show) — here, generously,
the error measured on the SAME iteration's band.

Kill criterion: build the tier only if the certified share is >= 60% AND the
projected step gain is >= 10%.  Projection: the lite pass is ~60% of a step; with
the tier every lite sample pays half an fp16 product and the uncertified share a full one:
gain = 0.60 x (1 - (0.5 + (1 - share))) of the step.

Usage: python tools/fp8_tier.py [kitti0 kitti5]   -> profiles/r5_fp8_tier.json
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)

import synthetic as S  # noqa: E402
from deep_sdf.workspace import fold_state  # noqa: E402
from oracle import dsr_oracle as O  # noqa: E402

E4M3_MAX = 448.0
LITE_SHARE_OF_STEP = 0.60


def e4m3(x):
    """Round to OCP e4m3fn (3 mantissa bits, bias 7, subnormals down to 2^-9, max 448), to nearest."""
    x = np.asarray(x, np.float64)
    a = np.abs(x)
    e = np.floor(np.log2(np.where(a > 0, a, 1.0)))
    e = np.maximum(e, -6.0)                      # below 2^-6: subnormal spacing 2^-9
    q = np.exp2(e - 3)
    r = np.round(a / q) * q                      # (numpy rounds half to even)
    return np.sign(x) * np.minimum(r, E4M3_MAX)


def pow2_scale(m, top):
    """power-of-two s with m * s <= top"""
    m = np.maximum(m, 1e-30)
    return np.exp2(np.floor(np.log2(top / m)))


class Fp8Decoder:
    def __init__(self, layers):
        self.layers = [(np.asarray(W, np.float64), np.asarray(b, np.float64)) for W, b in layers]
        self.q = {}
        for i in range(1, 8):                    # lin1..lin7 on fp8 MFMA; per-row scale
            W = self.layers[i][0]
            s = pow2_scale(np.abs(W).max(1, keepdims=True), E4M3_MAX / 2)
            self.q[i] = (e4m3(W * s), s)

    def forward(self, inp, tile=128):
        """products of two e4m3 values are exact in fp32 (8 significant bits), so an fp32 matmul of
        the quantized operands is the MFMA's exact-product, fp32-accumulate arithmetic"""
        n = inp.shape[0]
        x = inp
        h = np.maximum(x @ self.layers[0][0].T + self.layers[0][1], 0)
        for i in range(1, 8):
            if i == 4:
                h = np.concatenate([h, x], 1)
            Wq, sw = self.q[i]
            m = np.abs(h).reshape(-1, tile, h.shape[1]).max((1, 2)) if n % tile == 0 else None
            if m is None:
                pad = (-n) % tile
                hp = np.concatenate([h, np.zeros((pad, h.shape[1]))], 0)
                m = np.abs(hp).reshape(-1, tile, h.shape[1]).max((1, 2))
            sa = np.repeat(pow2_scale(m, E4M3_MAX / 2), tile)[:n, None]
            a = (e4m3(h * sa).astype(np.float32) @ Wq.T.astype(np.float32)).astype(np.float64) / (sa * sw.T)
            h = np.maximum((a + self.layers[i][1]).astype(np.float32), 0).astype(np.float64)
        y = h @ self.layers[8][0].T + self.layers[8][1]
        return np.tanh(y[:, 0])


def samples(f, e, M=50):
    """In-ball ray samples of recorded state e of fixture f, ray-major, + the ray index
    (optimizer.py:122-126, loss.py:71-82) and the lite-decoded mask (up to each ray's first
    sample with exact sdf <= -th: early ray termination)."""
    T = np.asarray(f["it_t_obj_cam"][e], np.float64)
    tco = np.linalg.inv(T)
    sc = np.linalg.det(tco[:3, :3]) ** (1.0 / 3.0)
    depths = np.linspace(tco[2, 3] - sc, tco[2, 3] + sc, M)
    rays = np.asarray(f["obj_rays"], np.float64)
    cam = rays[:, None, :] * depths[None, :, None]
    obj = cam @ T[:3, :3].T + T[:3, 3]
    inball = np.linalg.norm(obj, axis=-1) < 1.0
    return obj, inball


def main():
    names = sys.argv[1:] or ["kitti0", "kitti5"]
    th = 0.01
    layers = fold_state(S.make_decoder(1234), S.DEFAULT_SPECS)
    d64 = O.Decoder(layers)                      # fp32 reference: its 1e-7 error is nothing next to fp8's
    d8 = Fp8Decoder(layers)
    rows = []
    for name in names:
        f = np.load(os.path.join(REPO, "tests", "golden", f"f4_traj_{name}.npz"), allow_pickle=False)
        for e in range(int(f["n_iters_run"])):
            z = np.asarray(f["it_z"][e], np.float64)
            obj, inball = samples(f, e)
            ri, rj = np.nonzero(inball)
            q = obj[ri, rj]
            inp = np.concatenate([np.broadcast_to(z, (q.shape[0], 64)), q], 1)
            y = d64.forward(inp.astype(np.float32)).astype(np.float64)
            y8 = d8.forward(inp)
            # lite-decoded: every in-ball sample up to and including its ray's first full one
            full = y <= -th
            first_full = np.full(obj.shape[0], 10 ** 9)
            np.minimum.at(first_full, ri[full], rj[full])
            dec = rj <= first_full[ri]
            err = np.abs(y8 - y)
            band = dec & (np.abs(y) < th + 0.05)
            m8 = max(0.002, 4.0 * float(err[band].max())) if band.any() else 0.002
            cert = dec & ((y8 >= th + m8) | (y8 <= -th - m8))
            wrong = cert & (((y8 >= th + m8) & (y < th)) | ((y8 <= -th - m8) & (y > -th)))
            rows.append({"object": name, "iteration": e, "decoded": int(dec.sum()),
                         "max_err": float(err[dec].max()), "band_max_err": float(err[band].max()) if band.any() else 0.0,
                         "margin": m8, "certified_share": float(cert.sum() / max(1, dec.sum())),
                         "misclassified": int(wrong.sum())})
            print(json.dumps(rows[-1]), flush=True)
    share = float(np.sum([r["certified_share"] * r["decoded"] for r in rows]) / np.sum([r["decoded"] for r in rows]))
    gain = LITE_SHARE_OF_STEP * (1.0 - (0.5 + (1.0 - share)))
    out = {"rows": rows, "certified_share": share, "projected_step_gain": gain,
           "kill_criterion": "share >= 0.60 and projected step gain >= 0.10",
           "build": bool(share >= 0.60 and gain >= 0.10),
           "model": "OCP e4m3 weights (per-row pow2 scale) and activations (per 128-point tile and layer), exact "
                    "products, fp32 accumulation; fp32 lin0 / lin8; margin max(0.002, 4 x the iteration's band error)"}
    print(f"certified share {share:.3f}, projected step gain {gain:+.3f} -> build: {out['build']}")
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    with open(os.path.join(REPO, "profiles", "r5_fp8_tier.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
