"""Decoder precision of the fp32 and split-fp16 kernels vs an fp64 reference (diagnostic)."""
import os, sys
import numpy as np
sys.path.insert(0, "dsp-slam-rgbd_amd"); sys.path.insert(0, ".")
import synthetic as S
from deep_sdf.workspace import decoder_from_state, fold_state
from oracle import dsr_oracle as O
from reconstruct.optimizer import sdf_eval
state = S.make_decoder(1234)
dec = decoder_from_state(state, S.DEFAULT_SPECS)
layers = fold_state(state, S.DEFAULT_SPECS)
o64 = O.Decoder(layers, dtype=np.float64)
o32 = O.Decoder(layers)
rng = np.random.default_rng(0)
n = 20000
d = rng.standard_normal((n, 3)); d /= np.linalg.norm(d, axis=1, keepdims=True)
x = (d * (0.5 + 0.05 * rng.standard_normal((n, 1)))).astype(np.float32)
z = (0.05 * rng.standard_normal(64)).astype(np.float32)
inp = np.concatenate([np.broadcast_to(z, (n, 64)), x], 1)
y64, j64 = o64.forward_jac(inp.astype(np.float64))
y32, j32 = o32.forward_jac(inp)
def stats(name, y, j=None):
    e = np.abs(y - y64)
    msg = f"{name}: sdf max {e.max():.3e} rms {np.sqrt((e**2).mean()):.3e}"
    if j is not None:
        ej = np.abs(j - j64).max(axis=1) / np.abs(j64).max()
        msg += f" | jac rel p50 {np.median(ej):.3e} p99 {np.percentile(ej, 99):.3e} max {ej.max():.3e}"
    print(msg, flush=True)
stats("numpy fp32", y32, j32)
for fv, jv in [(6, 0), (12, 12)]:
    os.environ["DSR_FWD_VARIANT"] = str(fv); os.environ["DSR_JAC_VARIANT"] = str(jv)
    y = sdf_eval(dec, z, x)
    yj, j = sdf_eval(dec, z, x, with_jac=True)
    stats(f"gpu fwd V{fv}", y)
    stats(f"gpu jac V{jv}", yj, j)
