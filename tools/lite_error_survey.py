"""How large can the lite pass's error get?  A numpy emulation of the one-product fp16 lite
kernel (k_mlp_fwd_lite_st, DSR_LITE_VARIANT 1496: fp16(W) unscaled, fp16 activations, exact
products summed in fp32 from the bias, fp16 convert + ReLU per layer, lin0 and the lin8 dot
in fp32) against the fp64 decoder, over many decoders, codes and realistic in-ball ray
samples — the evidence behind the lite margin (margin = max(0.002, 4 x the
object's largest observed error), certain audit of th + 2 margin).

Usage: python tools/lite_error_survey.py [n_decoders]     (CPU, ~10 s per decoder x code)
Prints, per decoder (seed, hidden gain) and code scale: samples, max |lite - fp64|, its 99.99th
percentile, and the ratio of the max to the 0.002 margin floor and to 2 x that floor (the
audit shell's width beyond the band at the floor).
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


def lite_forward(layers, z, x):
    """The lite kernel's arithmetic (dsr_mlp_lite.hpp, LV 1496) on samples x (n, 3)."""
    W0, b0 = (np.asarray(a, np.float32) for a in layers[0])
    # lin0: code folded into the bias (fp32), xyz by fp32 fma in the kernel's order
    bias0 = (W0[:, :64].astype(np.float64) @ z.astype(np.float64) + b0).astype(np.float32)
    a = bias0[None, :] + ((x[:, 0:1] * W0[None, :, 64] + x[:, 1:2] * W0[None, :, 65]) + x[:, 2:3] * W0[None, :, 66])
    h = np.maximum(a, 0).astype(np.float16)
    W4, b4 = (np.asarray(a, np.float32) for a in layers[4])
    bias4 = (W4[:, 445:509].astype(np.float64) @ z.astype(np.float64) + b4).astype(np.float32)
    for li in range(1, 8):
        W, b = (np.asarray(a, np.float32) for a in layers[li])
        if li == 4:
            Wk = np.concatenate([W[:, :445], W[:, 509:512]], axis=1)       # h3 | xyz, code folded
            hin = np.concatenate([h, x.astype(np.float16)], axis=1)
            bias = bias4
        else:
            Wk, hin, bias = W, h, b
        acc = hin.astype(np.float64) @ Wk.astype(np.float16).astype(np.float64).T + bias   # exact products
        acc = acc.astype(np.float32)
        if li < 7:
            h = np.maximum(acc.astype(np.float16), np.float16(0))
        else:
            h7 = np.maximum(acc, 0)                                        # fp32 ReLU of the accumulator
    W8, b8 = (np.asarray(a, np.float32) for a in layers[8])
    return np.tanh(h7.astype(np.float64) @ W8[0].astype(np.float64) + b8[0])


def exact_forward(layers, z, x):
    inp = np.concatenate([np.broadcast_to(z, (x.shape[0], 64)), x], axis=1).astype(np.float64)
    h = inp
    for i, (W, b) in enumerate(layers):
        if i == 4:
            h = np.concatenate([h, inp], axis=1)
        h = h @ np.asarray(W, np.float64).T + b
        if i < 8:
            h = np.maximum(h, 0)
    return np.tanh(h[:, 0])


def samples(seed, n_obj=2):
    """In-ball ray samples of KITTI-like objects (the render pass's inputs), object frame."""
    from oracle import dsr_oracle as O

    out = []
    for i in range(n_obj):
        o = S.kitti_object(i, base_seed=seed)
        T = np.linalg.inv(o.t_cam_obj).astype(np.float32)
        s = np.float32(np.cbrt(np.linalg.det(o.t_cam_obj[:3, :3].astype(np.float64))))
        d = O.linspace_torch(np.float32(o.t_cam_obj[2, 3] - s), np.float32(o.t_cam_obj[2, 3] + s), 50)
        p = O.transform_points(o.rays[:, None, :] * d[:, None], T).reshape(-1, 3)
        out.append(p[np.linalg.norm(p, axis=1) < 1])
    return np.concatenate(out).astype(np.float32)


def main():
    n_dec = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    rng = np.random.default_rng(7)
    worst = 0.0
    print("decoder (seed, gain) | code scale | samples | max |lite - fp64| | p99.99 | max / 0.002 | band samples max")
    for k in range(n_dec):
        seed, gain = 1234 + 17 * k, (2.45, 2.0, 3.2)[k % 3]
        state = S.fit_last_layer_to_sphere(S.make_decoder_state(seed, hidden_gain=gain))
        layers = fold_state(state, S.DEFAULT_SPECS)
        x = samples(5000 + 11 * k)
        for cs in (0.0, 0.3, 1.0):
            z = (cs * rng.standard_normal(64)).astype(np.float32)
            e_all = []
            for c0 in range(0, x.shape[0], 20000):
                xs = x[c0:c0 + 20000]
                y = exact_forward(layers, z, xs)
                e_all.append((np.abs(lite_forward(layers, z, xs) - y), y))
            e = np.concatenate([a for a, _ in e_all])
            y = np.concatenate([b for _, b in e_all])
            band = np.abs(y) < 0.03
            worst = max(worst, float(e.max()))
            print(f"({seed}, {gain}) | {cs} | {e.size} | {e.max():.2e} | {np.quantile(e, 0.9999):.2e} | "
                  f"{e.max() / 0.002:.3f} | {e[band].max() if band.any() else 0:.2e} ({band.sum()})", flush=True)
    print(f"worst max error {worst:.2e} = {worst / 0.002:.3f} of the 0.002 margin floor "
          f"({worst / 0.004:.3f} of the audit shell's certain-audit width at the floor)")


if __name__ == "__main__":
    main()
