"""Per-phase cycle shares of k_mlp_jac16 from an exp_STAMP.so run.

Usage: python tools/jac_stamp_summary.py gpurun_out/stamp.txt [jac_stamp|fwd16_stamp]
(lines `jac_stamp|fwd16_stamp block wave tiles c0..c7` printed by blocks 0-3, waves 0 and 4;
fwd16: phase 6 = tanh + outputs, 7 = lin0 + mask queue, 0 = tile inputs)
"""
import sys

import numpy as np

NAMES = ["tile inputs / kept masks", "GEMMs", "epilogue compute", "scale exchange (barrier)",
         "split writes", "post-write barrier", "J tail", "other (lin0, g7, lin7, lin0^T)"]
KEY = sys.argv[2] if len(sys.argv) > 2 else "jac_stamp"
rows = [ln.split()[1:] for ln in open(sys.argv[1]) if ln.startswith(KEY + " ")]
a = np.array(rows, dtype=np.float64)
if a.shape[1] > 11:   # fwd16_stamp: 12 phases
    NAMES = ["tile inputs", "GEMMs", "epilogue compute", "scale exchange (barrier)", "split writes",
             "post-write barrier", "outputs' final atomic + barrier", "lin0 + mask queue",
             "lin7 epilogue + mask store", "pre-tail barrier", "tail: sum + tanh", "tail: checks + stores"]
for w in (0, 4):
    sel = a[a[:, 1] == w]
    if not len(sel):
        continue
    tot = sel[:, 3:3 + len(NAMES)].sum()
    print(f"wave {w}: {len(sel)} block-launches, {sel[:, 2].sum():.0f} tiles, "
          f"{tot / max(1, sel[:, 2].sum()):.0f} cycles per tile")
    for n, v in zip(NAMES, sel[:, 3:3 + len(NAMES)].sum(0) / tot):
        print(f"   {n:34s} {v:.3f}")
