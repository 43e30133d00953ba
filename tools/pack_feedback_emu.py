"""Numpy emulation of the split packs' weight representation in the BACKWARD chain (CPU): the
Jacobian d sdf / d[code, xyz] of the bench decoder with every W_l^T replaced by hi + lo of its
split pack, against fp64, for three ways of choosing lo (dsr_api.hip: pack_frag16):
  nearest   lo = fp16(W 2^sw - hi)
  mean      error feedback along each row against the mean of the GEMM's inputs at 256 probe
            points (round 5's first rule)
  moments   greedy error feedback against the inputs' second moments: keep
            sum_p ((hi + lo - W 2^sw) . g_p)^2 small (the shipped rule)
Products exact, so only the weights' rounded-away tails show.  Reported as tools/bias_probe.py
does: the systematic part (per-component mean error over 40k points on a shell around the
surface, in units of the component's mean |J|, RMS over components) and the random part.

usage: python tools/pack_feedback_emu.py     (~5 min, single-threaded numpy)
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
from oracle import dsr_oracle as O  # noqa: E402


def f16(v):
    return v.astype(np.float16).astype(np.float64)


def split(W, mode, C=None, gbar=None):
    """hi + lo of W (rows r, k along axis 1) with lo chosen by `mode`"""
    s = 14 - np.frexp(np.abs(W).max())[1]
    xs = W * 2.0 ** s
    hi = f16(xs)
    r = xs - hi
    lo = f16(r)
    if mode != "nearest":
        l16 = lo.astype(np.float16)
        up = np.nextafter(l16, np.float16(np.inf)).astype(np.float64)
        dn = np.nextafter(l16, np.float16(-np.inf)).astype(np.float64)
        other = np.where(lo < r, up, dn)
        acc = np.zeros(W.shape[0]) if mode == "mean" else np.zeros(W.shape)
        for j in range(W.shape[1]):
            d1, d2 = lo[:, j] - r[:, j], other[:, j] - r[:, j]
            if mode == "mean":
                use = np.abs(acc + d2 * gbar[j]) < np.abs(acc + d1 * gbar[j])
            else:       # acc = e C (e: the row's error so far), cost change 2 d (eC)_j + d^2 C_jj
                use = 2 * d2 * acc[:, j] + d2 * d2 * C[j, j] < 2 * d1 * acc[:, j] + d1 * d1 * C[j, j]
            use &= lo[:, j] != r[:, j]
            lo[:, j] = np.where(use, other[:, j], lo[:, j])
            d = lo[:, j] - r[:, j]
            if mode == "mean":
                acc = acc + d * gbar[j]
            else:
                acc += d[:, None] * C[j][None, :]
    return (hi + lo) * 2.0 ** -s


def main():
    layers = fold_state(S.make_decoder(1234), S.DEFAULT_SPECS)
    D = O.Decoder(layers, dtype=np.float64)
    rng = np.random.default_rng(0)
    n = 40000
    d = rng.standard_normal((n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    x = d * (0.5 + 0.02 * rng.standard_normal((n, 1)))
    inp = np.concatenate([np.zeros((n, 64)), x], 1)
    y, masks, _ = D.forward(inp, keep_masks=True, keep_pre=True)

    def jac(Wt):
        g = (1 - y * y)[:, None]
        gin = np.zeros_like(inp)
        for i in range(8, -1, -1):
            g = g @ (D.layers[i][0] if i == 8 else Wt[i])
            if i == 4:
                gin = gin + g[:, -67:]
                g = g[:, :-67]
            if i > 0:
                g = np.where(masks[i - 1], g, 0.0)
        return g + gin

    j64 = jac({i: D.layers[i][0] for i in range(8)})
    pp = rng.uniform(-1, 1, (1024, 3))
    pp = pp[(pp ** 2).sum(1) < 1][:256]
    yy, mk, _ = D.forward(np.concatenate([np.zeros((len(pp), 64)), pp], 1), keep_masks=True, keep_pre=True)
    g = (1 - yy * yy)[:, None]
    gm, C = {}, {}
    for i in range(8, -1, -1):
        if i < 8:
            g = np.where(mk[i], g, 0.0)
            gm[i], C[i] = g.mean(0), g.T @ g / g.shape[0]
        g = g @ D.layers[i][0]
        if i == 4:
            g = g[:, :-67]
    for mode in ("nearest", "mean", "moments"):
        Wt = {i: split(np.asarray(D.layers[i][0], np.float32).astype(np.float64).T, mode, C.get(i), gm.get(i)).T
              for i in range(8)}
        e = (jac(Wt) - j64) / np.abs(j64).mean(0)
        print(f"{mode:8s}: Jacobian systematic {np.sqrt((e.mean(0) ** 2).mean()):.2e} of mean |J| "
              f"(code {np.sqrt((e[:, :64].mean(0) ** 2).mean()):.2e}, xyz {np.sqrt((e[:, 64:].mean(0) ** 2).mean()):.2e}),"
              f" random {np.sqrt(e.var(0).mean()):.2e}", flush=True)


if __name__ == "__main__":
    main()
