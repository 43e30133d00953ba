"""Signed (systematic) error of the decoder sdf and Jacobian against fp64 on surface-like points
(diagnostic; GPU box): numpy fp32, the fp32-MFMA kernels (variant 0) and the split-fp16 kernels
(12).  A bias — the same sign on every point — adds up coherently in b = sum J r (optimizer.py:
163-169) where random rounding averages out."""
import os
import sys

import numpy as np

sys.path.insert(0, "dsp-slam-rgbd_amd")
sys.path.insert(0, ".")
import synthetic as S  # noqa: E402
from deep_sdf.workspace import decoder_from_state, fold_state  # noqa: E402
from oracle import dsr_oracle as O  # noqa: E402
from reconstruct.optimizer import sdf_eval  # noqa: E402

os.environ["DSR_TEST_HOOKS"] = "1"
import time  # noqa: E402
state = S.make_decoder(1234)
t0 = time.perf_counter()
dec = decoder_from_state(state, S.DEFAULT_SPECS)
print(f"decoder load {time.perf_counter() - t0:.3f} s (qualification {dec.info['probe_ms']:.1f} ms)", flush=True)
layers = fold_state(state, S.DEFAULT_SPECS)
o64 = O.Decoder(layers, dtype=np.float64)
o32 = O.Decoder(layers)
rng = np.random.default_rng(0)
n = 40000
d = rng.standard_normal((n, 3))
d /= np.linalg.norm(d, axis=1, keepdims=True)
x = (d * (0.5 + 0.02 * rng.standard_normal((n, 1)))).astype(np.float32)
for zs in (0.0, 0.05):
    z = (zs * rng.standard_normal(64)).astype(np.float32)
    inp = np.concatenate([np.broadcast_to(z, (n, 64)), x], 1)
    y64, j64 = o64.forward_jac(inp.astype(np.float64))
    y32, j32 = o32.forward_jac(inp)
    jn = np.abs(j64).mean(0)

    def stats(name, y, j):
        e = y.astype(np.float64) - y64
        ej = (j.astype(np.float64) - j64) / jn          # per component, in units of its mean |J|
        print(f"code scale {zs} {name}: sdf mean {e.mean():+.2e} (SE {e.std() / np.sqrt(n):.1e}) rms {np.sqrt((e * e).mean()):.2e}"
              f" | J code mean {ej[:, :64].mean():+.2e} rms {np.sqrt((ej[:, :64] ** 2).mean()):.2e}"
              f" J xyz mean {ej[:, 64:].mean():+.2e} rms {np.sqrt((ej[:, 64:] ** 2).mean()):.2e}"
              f" | sum_p J*e_sdf / sum|J||e| code {np.abs((j64[:, :64] * e[:, None]).sum(0)).max() / (np.abs(j64[:, :64]) * np.abs(e)[:, None]).sum(0).max():.3f}",
              flush=True)
        # systematic part of the Jacobian error per component (its mean over points), RMS over the
        # components, against the same for the random part — kink-flip points excluded
        jr = np.abs(j.astype(np.float64) - j64).max(1) / np.abs(j64).max()
        ok = jr < 1e-5
        ejc = (j.astype(np.float64) - j64)[ok] / np.abs(j64[ok]).mean(0)
        print(f"    J error per component (kinks excluded): systematic rms {np.sqrt((ejc.mean(0) ** 2).mean()):.2e}"
              f" (code {np.sqrt((ejc[:, :64].mean(0) ** 2).mean()):.2e}, xyz {np.sqrt((ejc[:, 64:].mean(0) ** 2).mean()):.2e}),"
              f" random rms {np.sqrt(ejc.var(0).mean()):.2e}", flush=True)
        print(f"    J kink flips (per-point max |dJ| > 1e-5 max|J|): {np.mean(jr > 1e-5):.4f} of points; > 1e-6: {np.mean(jr > 1e-6):.4f}", flush=True)
        cbk = (np.arange(n) % 64) // 16          # the point's 16-point block in its 64-point tile
        print("    sdf mean by point block cb 0..3: " + " ".join(f"{e[cbk == k].mean():+.2e}" for k in range(4)), flush=True)
    stats("numpy fp32", y32, j32)
    for fv, jv in [(0, 0), (12, 12)]:
        os.environ["DSR_FWD_VARIANT"] = str(fv)
        os.environ["DSR_JAC_VARIANT"] = str(jv)
        yj, j = sdf_eval(dec, z, x, with_jac=True)
        stats(f"gpu jac V{jv}", yj, j)
