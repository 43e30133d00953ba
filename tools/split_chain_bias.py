"""Bias of one split-fp16 GEMM output the way the decoder kernels accumulate it (diagnostic, GPU
box): 16 k steps x (al.bh, ah.bl, ah.bh) on v_mfma_f32_16x16x32_f16 into one accumulator,
operands like a decoder layer's — weights N(0, 1) scaled to |W| < 2^14 and split hi/lo (A),
ReLU'd activations (half zeros, positive) scaled and split (B) — against the exact value of the
same split operands.  Reports the mean error relative to |exact| (toward -inf: err / |exact|) and
its toward-zero part (err * sign(exact) / |exact|), with the weights as they are and negated."""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libmfma_numerics.so"))
FP = ctypes.POINTER(ctypes.c_float)


def split(x, s):
    x = (x * 2.0 ** s).astype(np.float32)
    h = x.astype(np.float16)
    lo = (x - h.astype(np.float32)).astype(np.float16)
    return h, lo


rng = np.random.default_rng(11)
T = 2048
W = rng.standard_normal((T, 16, 512)).astype(np.float32)
H = np.maximum(rng.standard_normal((T, 512, 16)), 0).astype(np.float32) * np.exp2(rng.uniform(-3, 0, (T, 1, 16))).astype(np.float32)
for (name, sg), mode in [(c, m) for m in (0, 1, 2) for c in (("weights as packed", 1.0), ("weights negated", -1.0))]:
    name = f"chain mode {mode} ({('one chain', 'step sums + VALU add', 'lo from zero + VALU add')[mode]}), {name}"
    Wh, Wl = split(sg * W / np.abs(W).max() * 0.99, 14)
    Hh, Hl = split(H / H.max(), 13)
    A = np.ascontiguousarray(np.stack([Wh, Wl], 1))
    B = np.ascontiguousarray(np.stack([Hh, Hl], 1))
    D = np.zeros((T, 16, 16), np.float32)
    assert lib.split_chain(ctypes.c_void_p(A.ctypes.data), ctypes.c_void_p(B.ctypes.data), D.ctypes.data_as(FP), T, mode) == 0
    a = Wh.astype(np.float64), Wl.astype(np.float64)
    b = Hh.astype(np.float64), Hl.astype(np.float64)
    ex = np.einsum("tik,tkj->tij", a[1], b[0]) + np.einsum("tik,tkj->tij", a[0], b[1]) + np.einsum("tik,tkj->tij", a[0], b[0])
    # unit: the output's typical magnitude sqrt(sum_k (a_k b_k)^2) (no cancellation blow-up)
    u = np.sqrt(np.einsum("tik,tkj->tij", a[0] ** 2, b[0] ** 2))
    ok = u > 0
    e = (D.astype(np.float64) - ex)[ok] / u[ok]
    sz = np.sign(ex[ok])
    se = e.std() / np.sqrt(e.size)
    print(f"{name}: mean err/u {e.mean():+.3e} (SE {se:.1e}), toward-zero part {(e * sz).mean():+.3e}, rms {np.sqrt((e * e).mean()):.3e}"
          f" | fp32 RNE of exact: rms {np.sqrt((((ex.astype(np.float32) - ex)[ok] / u[ok]) ** 2).mean()):.3e}", flush=True)
