"""Would a TWO-product fp16 split do for the exact pass and the Jacobian?  

The split kernels carry every GEMM operand x as hi + lo fp16 pieces under a
power-of-two scale and form A.B = Ah.Bh + Ah.Bl + Al.Bh (3 MFMA products, ~22 significant bits
per operand).  Dropping one cross product would cut the exact pass's and the Jacobian's MFMA
work by a third.  This script emulates, in numpy, the decoder forward and input-Jacobian with
the kernels' operand handling —

* weights: one power-of-two scale per matrix (max|W| 2^sw < 2^14), pieces fp16;
* activations / back-propagated gradients: one power-of-two scale per 64-point tile and layer
  from the tile's max, pieces fp16;
* products exact, sums in fp64 (the MFMA's fp32 accumulation adds ~1e-7 relative on top);
* lin0 (3 inputs, code folded into the bias) and lin8 (a dot product) in fp32 as in the kernels

— for four product sets: "3prod" (the shipped split), "2prod_W16" (Wh.(Hh + Hl): weights at
fp16 precision), "2prod_H16" ((Wh + Wl).Hh: activations at fp16 precision) and "1prod"
(Wh.Hh, the lite pass), and checks sdf and Jacobian against golden F1 (the reference's own
fp32 values, tests/golden/f1_decoder_full.npz) at the parity suite's tolerances: sdf <= 2e-5,
Jacobian <= 1e-4 x max|J| (a few ReLU-kink points excepted, conftest.assert_jac_close).

Usage: python tools/two_product_split.py      (CPU, ~1 min; prints one line per product set)
"""
from __future__ import annotations

import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)

import synthetic as S  # noqa: E402
from deep_sdf.workspace import fold_state  # noqa: E402

TILE = 64


def _pow2_scale(mx, top):
    """Exponent s with mx * 2^s < 2^top (as the kernels' act_scale_exp / pack_frag16)."""
    if mx <= 0 or not np.isfinite(mx):
        return 0
    return top - int(np.frexp(mx)[1])


def split(x, s):
    xs = np.asarray(x, np.float64) * 2.0 ** s
    hi = xs.astype(np.float16).astype(np.float64)
    lo = (xs - hi).astype(np.float16).astype(np.float64)
    return hi, lo


def gemm(W, H, mode):
    """W (out, k) . H (k, n) with n a multiple of TILE, per-tile activation scales."""
    sw = _pow2_scale(np.abs(W).max(), 14)
    Wh, Wl = split(W, sw)
    out = np.zeros((W.shape[0], H.shape[1]))
    for t in range(0, H.shape[1], TILE):
        Ht = H[:, t:t + TILE]
        sa = _pow2_scale(np.abs(Ht).max(), 15)
        Hh, Hl = split(Ht, sa)
        if mode == "3prod":
            acc = Wh @ Hh + Wh @ Hl + Wl @ Hh
        elif mode == "2prod_W16":
            acc = Wh @ (Hh + Hl)
        elif mode == "2prod_H16":
            acc = (Wh + Wl) @ Hh
        elif mode == "1prod":
            acc = Wh @ Hh
        else:
            acc = (np.asarray(W, np.float64) * 2.0 ** sw) @ (np.asarray(Ht, np.float64) * 2.0 ** sa)
        out[:, t:t + TILE] = acc * 2.0 ** (-(sw + sa))
    return out.astype(np.float32)


def forward_jac(layers, z, x, mode):
    """sdf (n,) and d sdf / d[z, x] (n, 67) with every GEMM of lin1..lin7 (and the backward
    GEMMs of lin7^T..lin0^T) through ``gemm``."""
    n = x.shape[0]
    npad = (n + TILE - 1) // TILE * TILE
    inp = np.zeros((npad, 67), np.float32)
    inp[:n, :64] = z
    inp[:n, 64:] = x
    W0, b0 = layers[0]
    h = np.maximum(inp @ W0.T.astype(np.float32) + b0, 0).astype(np.float32)         # lin0, fp32
    masks, hs = [h > 0], []
    for li in range(1, 8):
        W, b = layers[li]
        hin = h
        if li == 4:
            hin = np.concatenate([h, inp], axis=1)
        hs.append(hin)
        pre = gemm(W, hin.T, mode).T + b
        h = np.maximum(pre, 0).astype(np.float32)
        masks.append(pre > 0)
    W8, b8 = layers[8]
    s = (h @ W8[0].astype(np.float32) + b8[0]).astype(np.float32)
    y = np.tanh(s)
    g = ((1.0 - y * y)[:, None] * W8[0][None, :]).astype(np.float32)                  # d/d h7
    grad_in = np.zeros((npad, 67), np.float32)
    for li in range(7, 0, -1):
        W, _ = layers[li]
        g = np.where(masks[li], g, 0).astype(np.float32)                              # ReLU' of lin li
        gin = gemm(W.T, g.T, mode).T                                                   # d/d input of lin li
        if li == 4:
            grad_in += gin[:, 445:]
            gin = gin[:, :445]
        g = gin
    g = np.where(masks[0], g, 0).astype(np.float32)
    grad_in += gemm(W0.T, g.T, mode).T
    return y[:n], grad_in[:n]


def jac_check(j, jref, tol=1e-4, loose=5e-2, frac=0.01):
    scale = max(1.0, float(np.abs(jref).max()))
    per_pt = np.abs(np.asarray(j, np.float64) - jref).max(axis=1) / scale
    n_bad = int((per_pt > tol).sum())
    ok = n_bad <= max(2, int(frac * per_pt.shape[0])) and per_pt.max() <= loose
    return ok, float(np.median(per_pt)), float(np.quantile(per_pt, 0.99)), n_bad


def main():
    f = np.load(os.path.join(REPO, "tests", "golden", "f1_decoder_full.npz"), allow_pickle=False)
    layers = [(np.asarray(W, np.float32), np.asarray(b, np.float32))
              for W, b in fold_state(S.make_decoder(1234), S.DEFAULT_SPECS)]
    z, x = f["z"].astype(np.float32), f["x"].astype(np.float32)
    print(f"F1: {x.shape[0]} points; tolerances sdf <= 2e-5, J <= 1e-4 x max|J| ({np.abs(f['jac']).max():.3f})")
    for mode in ("fp64", "3prod", "2prod_W16", "2prod_H16", "1prod"):
        y, J = forward_jac(layers, z, x, mode)
        e_sdf = float(np.abs(y - f["sdf"]).max())
        ok, med, q99, nbad = jac_check(J, f["jac"])
        verdict = "PASS" if (e_sdf <= 2e-5 and ok) else "FAIL"
        print(f"{mode:10s} sdf max err {e_sdf:.2e} (rms {np.sqrt(np.mean((y - f['sdf']) ** 2)):.1e})  "
              f"J rel err median {med:.1e} p99 {q99:.1e} points > 1e-4: {nbad}  -> {verdict}", flush=True)


if __name__ == "__main__":
    main()
