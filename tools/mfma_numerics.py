"""How gfx950's MFMA rounds (diagnostic): D = A.B + C on v_mfma_f32_16x16x32_f16 (one and two
chained k steps) and v_mfma_f32_16x16x4_f32, against the exact sums (Python fractions) rounded
to nearest-even and toward zero.  Build: hipcc --offload-arch=gfx950 -O2 -shared -fPIC
tools/mfma_numerics.hip -o tools/libmfma_numerics.so.  Run on the GPU box."""
import ctypes
import os
import sys
from fractions import Fraction

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libmfma_numerics.so"))
P = ctypes.c_void_p


def f32_round(x: Fraction, mode: str) -> np.float32:
    """x rounded to fp32 (normal range) to nearest-even ('rne') or toward zero ('rtz')."""
    if x == 0:
        return np.float32(0)
    s = -1 if x < 0 else 1
    a = abs(x)
    e = a.numerator.bit_length() - a.denominator.bit_length()
    if Fraction(2) ** e > a:
        e -= 1
    q = a / Fraction(2) ** (e - 23)           # in [2^23, 2^24)
    n, r = divmod(q.numerator, q.denominator)
    if mode == "rne":
        rem = Fraction(r, q.denominator)
        if rem > Fraction(1, 2) or (rem == Fraction(1, 2) and n % 2 == 1):
            n += 1
    return np.float32(s * n * 2.0 ** (e - 23))


def run(mode, n_trial, rng, cscale, spread):
    if mode == 2:
        A = rng.standard_normal((n_trial, 16, 4)).astype(np.float32)
        B = rng.standard_normal((n_trial, 4, 16)).astype(np.float32)
        K = 4
    else:
        K = 64 if mode == 1 else 32
        A = (rng.standard_normal((n_trial, 16, K)) * 2.0 ** rng.integers(-spread, spread + 1, (n_trial, 16, K))).astype(np.float16)
        B = rng.standard_normal((n_trial, K, 16)).astype(np.float16)
    C = (rng.standard_normal((n_trial, 16, 16)) * cscale).astype(np.float32)
    Ct = np.ascontiguousarray(C)                    # row-major [i][j], as the probe indexes C and D
    D = np.zeros_like(Ct)
    Ac, Bc = np.ascontiguousarray(A), np.ascontiguousarray(B)
    assert lib.probe(P(Ac.ctypes.data), P(Bc.ctypes.data), Ct.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                     D.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n_trial, mode) == 0
    DUMP.append(dict(mode=mode, A=A, B=B, C=C, D=D))
    stats = {"rne": 0, "rtz": 0, "chain_rne": 0, "fma_chain": 0, "none": 0}
    ulp_err = []
    for t in range(n_trial):
        for i in range(16):
            for j in range(16):
                prods = [Fraction(float(A[t, i, k])) * Fraction(float(B[t, k, j])) for k in range(K)]
                ex = sum(prods, Fraction(float(C[t, i, j])))
                d = D[t, i, j]
                rne, rtz = f32_round(ex, "rne"), f32_round(ex, "rtz")
                # k-step chain with one RNE rounding per 32-deep step (mode 1)
                ch = Fraction(float(C[t, i, j]))
                for s0 in range(0, K, 32):
                    ch = Fraction(float(f32_round(ch + sum(prods[s0:s0 + 32], Fraction(0)), "rne")))
                hit = False
                if d == rne:
                    stats["rne"] += 1
                    hit = True
                if d == rtz:
                    stats["rtz"] += 1
                    hit = True
                if np.float32(float(ch)) == d:
                    stats["chain_rne"] += 1
                    hit = True
                fc = Fraction(float(C[t, i, j]))         # one RNE rounding per product (an fma chain)
                for p_ in prods:
                    fc = Fraction(float(f32_round(fc + p_, "rne")))
                if np.float32(float(fc)) == d:
                    stats["fma_chain"] += 1
                    hit = True
                if not hit:
                    stats["none"] += 1
                if ex != 0:
                    u = abs(float(ex)) * 2.0 ** -23
                    # signed toward |exact|: negative = rounded toward zero
                    ulp_err.append(float((Fraction(float(d)) - ex)) / u * (1 if ex > 0 else -1))
    u = np.array(ulp_err)
    print(f"mode {mode} K {K} cscale {cscale} spread {spread}: {n_trial * 256} outputs; equal to RNE {stats['rne']}, "
          f"RTZ {stats['rtz']}, per-step RNE chain {stats['chain_rne']}, fma chain {stats['fma_chain']}, none {stats['none']}; "
          f"error in ulps of |exact|: mean {u.mean():+.3f} rms {np.sqrt((u * u).mean()):.3f} max {np.abs(u).max():.2f}",
          flush=True)


if __name__ == "__main__":
    rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
    DUMP = []
    for mode in (0, 1, 2):
        for cscale in (0.0, 1.0, 30.0):
            run(mode, 16, rng, cscale, 0)
    run(0, 16, rng, 1.0, 6)
    run(1, 16, rng, 1.0, 6)
    run(0, 64, rng, 0.0, 3)
    run(0, 64, rng, 8.0, 0)
    out = os.path.join(HERE, "..", "gpurun_out", "mfma_numerics.npz")
    np.savez_compressed(out, **{f"{k}{i}": v for i, d in enumerate(DUMP) for k, v in d.items()})
