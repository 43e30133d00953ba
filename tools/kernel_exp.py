"""Time single-iteration batches per kernel variant (identical inputs for every variant).

Usage (GPU box): python tools/kernel_exp.py --fwd 12 44 76 [--jac 12 28] [--rounds 5]
Each run is ONE GN iteration over 64 KITTI-like objects, so the fwd/jac launches see the
same tiles whatever a variant computes — timing experiments with invalid results (fwd
variants 44/76: reduced / no epilogue) stay comparable.  Prints median ms per launch and
the fp32-equivalent TFLOP/s from the kernels' own point counts.
"""
import argparse, ctypes as C, os, sys
import numpy as np
sys.path.insert(0, "dsp-slam-rgbd_amd"); sys.path.insert(0, ".")
import synthetic as S
from deep_sdf.workspace import decoder_from_state
from reconstruct import _libdsr as L
import bench

ap = argparse.ArgumentParser()
ap.add_argument("--fwd", nargs="*", type=int, default=[12])
ap.add_argument("--jac", nargs="*", type=int, default=[12])
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--objects", type=int, default=64)
a = ap.parse_args()
dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
cfg = dict(S.KITTI_OPTIM, joint_optim=dict(S.KITTI_OPTIM["joint_optim"], num_iterations=1))
batch, keep = bench.make_batch(dec, L.optim_params(cfg), a.objects, 1000)
lib, ctx = dec.ctx.lib, dec.ctx
outs = (L.ObjectOut * a.objects)()
combos = [(f, j) for f in a.fwd for j in a.jac]
res = {k: [] for k in combos}
for r in range(a.rounds):
    for f, j in combos:
        os.environ["DSR_FWD_VARIANT"] = str(f)
        os.environ["DSR_JAC_VARIANT"] = str(j)
        ctx.check(lib.dsr_batch_run(batch), "run")
        ctx.check(lib.dsr_batch_download(batch, outs), "dl")
        st = L.Stats(); ctx.check(lib.dsr_batch_stats(batch, C.byref(st)), "stats")
        res[(f, j)].append((st.fwd_ms, st.jac_ms,
                            2 * bench.FWD_MAC * st.fwd_points / (st.fwd_ms * 1e-3) / 1e12,
                            2 * (bench.FWD_MAC + bench.BWD_MAC) * st.jac_points / (st.jac_ms * 1e-3) / 1e12,
                            st.fwd_points, st.jac_points, st.refine_ms, st.refine_points))
for k in combos:
    x = np.median(np.array(res[k]), axis=0)
    print(f"fwd V{k[0]:3d} {x[0]:7.2f} ms {x[2]:6.1f} TF | refine {x[6]:6.2f} ms {int(x[7])} pts | "
          f"jac V{k[1]:3d} {x[1]:6.2f} ms {x[3]:6.1f} TF | pts {int(x[4])} / {int(x[5])}")
