"""Per-phase cycle shares of the staggered lite kernel from an exp_STAMP.so run.

Usage: python tools/stamp_summary.py gpurun_out/stamp.txt
(lines `lite_stamp block wave tiles c0..c8` printed by blocks 0-3, waves 0 and 4)
"""
import sys

import numpy as np

NAMES = ["tile inputs (+cE/cT waits)", "lin0", "epilogue waits (cRlo/cRhi)", "stores + signal",
         "GEMM pre-waits (cH/cP)", "GEMM (incl. A's step-7 wait)", "epilogue compute", "lin7 + classify"]
rows = [ln.split()[1:] for ln in open(sys.argv[1]) if ln.startswith("lite_stamp")]
a = np.array(rows, dtype=np.float64)
for w in (0, 4):
    sel = a[a[:, 1] == w]
    if not len(sel):
        continue
    tot = sel[:, 3:11].sum()
    print(f"wave {w} ({'group A' if w < 4 else 'group B'}): {len(sel)} block-launches, "
          f"{sel[:, 3:11].sum(1).mean() / max(1, sel[:, 2].mean()):.0f} cycles per tile")
    for n, v in zip(NAMES, sel[:, 3:11].sum(0) / tot):
        print(f"   {n:32s} {v:.3f}")
    if w == 0:
        print(f"   {'(of GEMM: step-7 wait for B)':32s} {sel[:, 11].sum() / tot:.3f}")
