"""Signed error of v_mfma_f32_16x16x32_f16 (diagnostic, GPU box): D = A.B + C against the float64
sum, in units of ulp(|C|) and of ulp(max |term|), for the operand regimes the split-fp16 kernels
(dsr_mlp16.hpp) produce: the hi.hi product into a running accumulator, the lo corrections
(2^-11 of it) into that accumulator, and products into a zero accumulator.
Needs tools/libmfma_numerics.so (tools/mfma_numerics.py)."""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libmfma_numerics.so"))
FP = ctypes.POINTER(ctypes.c_float)


def mfma(A, B, C):
    A = np.ascontiguousarray(A.astype(np.float16))
    B = np.ascontiguousarray(B.astype(np.float16))
    C = np.ascontiguousarray(C.astype(np.float32))
    D = np.zeros_like(C)
    assert lib.probe(ctypes.c_void_p(A.ctypes.data), ctypes.c_void_p(B.ctypes.data), C.ctypes.data_as(FP),
                     D.ctypes.data_as(FP), A.shape[0], 0) == 0
    ex = np.einsum("tik,tkj->tij", A.astype(np.float64), B.astype(np.float64)) + C.astype(np.float64)
    return D.astype(np.float64), ex, A, B, C


def ulp(x):
    return np.spacing(np.abs(x).astype(np.float32)).astype(np.float64)


rng = np.random.default_rng(5)
T = 512
for name, cs, ps in [("products ~1, C = 0", 0.0, 1.0), ("products ~1, C ~ 1", 1.0, 1.0),
                     ("products ~1, C ~ 16", 16.0, 1.0), ("lo products 2^-11, C ~ 16", 16.0, 2.0 ** -11),
                     ("lo products 2^-11, C ~ 1", 1.0, 2.0 ** -11), ("products 2^-6, C ~ 1", 1.0, 2.0 ** -6)]:
    A = rng.standard_normal((T, 16, 32)) * ps
    B = rng.standard_normal((T, 32, 16))
    C = rng.standard_normal((T, 16, 16)) * cs
    D, ex, A16, B16, C32 = mfma(A, B, C)
    e = D - ex
    tmax = np.maximum(np.abs(C32).astype(np.float64), np.abs(np.einsum("tik,tkj->tikj", A16.astype(np.float64),
                                                                     B16.astype(np.float64))).max(2))
    eu = e / ulp(tmax)
    er = e / ulp(ex)
    print(f"{name:28s}: err/ulp(max term) mean {eu.mean():+.4f} (SE {eu.std() / np.sqrt(eu.size):.4f}) rms {np.sqrt((eu ** 2).mean()):.3f}"
          f" | err/ulp(result) mean {er.mean():+.4f} rms {np.sqrt((er ** 2).mean()):.3f} | frac D>exact {np.mean(e > 0):.3f} D<exact {np.mean(e < 0):.3f}",
          flush=True)
