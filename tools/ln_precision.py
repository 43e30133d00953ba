"""Decoder precision vs fp64 truth for the variant decoders (GPU): sdf and Jacobian errors of the
GPU (split-fp16) and of the reference's fp32 (golden F17) against the fp64 oracle, per variant.
    python tools/ln_precision.py"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dsp-slam-rgbd_amd"), os.path.join(REPO, "tests")]

import synthetic as S  # noqa: E402
from oracle import dsr_oracle as O  # noqa: E402
from test_oracle_golden import _variant_specs  # noqa: E402


def main():
    from deep_sdf.workspace import decoder_from_state
    from reconstruct.optimizer import sdf_eval

    f = np.load(os.path.join(REPO, "tests", "golden", "f17_variants.npz"))
    for v in ("plain", "tanh", "xyz", "ln"):
        sp = _variant_specs(v)
        st = S.make_decoder(1234, sp)
        d64 = O.Decoder.from_state(st, sp, dtype=np.float64)
        z, x = f[v + "_z"], f[v + "_x"]
        y64, j64 = d64.forward_jac(np.concatenate([np.broadcast_to(z, (256, 64)), x], 1).astype(np.float64))
        y, j = sdf_eval(decoder_from_state(st, sp), z, x, with_jac=True)
        sc = np.abs(j64).max()
        print(f"{v}: sdf err gpu {np.abs(y - y64).max():.2e} ref {np.abs(f[v + '_sdf'] - y64).max():.2e} | "
              f"J err/max gpu med {np.median(np.abs(j - j64).max(1)) / sc:.2e} max {np.abs(j - j64).max() / sc:.2e} "
              f"ref med {np.median(np.abs(f[v + '_jac'] - j64).max(1)) / sc:.2e} max {np.abs(f[v + '_jac'] - j64).max() / sc:.2e}",
              flush=True)


if __name__ == "__main__":
    main()
