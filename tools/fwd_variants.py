"""A/B the k_mlp_fwd variants in ONE process, interleaved (cdna guide §5.4 rule 24).

Usage (GPU box): python tools/fwd_variants.py [variants...] [--objects 64] [--rounds 3]
Prints per-variant fwd kernel ms/launch (HIP events), batch ms, and checks that every
variant returns bitwise-identical results (the variants only change scheduling).
"""
import argparse, ctypes as C, os, sys, time
import numpy as np
sys.path.insert(0, "dsp-slam-rgbd_amd"); sys.path.insert(0, ".")
import synthetic as S
from deep_sdf.workspace import decoder_from_state
from reconstruct import _libdsr as L
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)) + "/..")
import bench

ap = argparse.ArgumentParser()
ap.add_argument("variants", nargs="*", type=int, default=[0, 1, 2, 3, 6, 7])
ap.add_argument("--objects", type=int, default=64)
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
params = L.optim_params(S.KITTI_OPTIM)
batch, keep = bench.make_batch(dec, params, a.objects, 1000)
lib, ctx = dec.ctx.lib, dec.ctx
outs = (L.ObjectOut * a.objects)()
res = {v: [] for v in a.variants}
ref = {}
for r in range(a.rounds):
    for v in a.variants:
        os.environ["DSR_FWD_VARIANT"] = str(v)
        t0 = time.perf_counter()
        ctx.check(lib.dsr_batch_run(batch), "run")
        ctx.check(lib.dsr_batch_download(batch, outs), "dl")
        dt = time.perf_counter() - t0
        st = L.Stats(); ctx.check(lib.dsr_batch_stats(batch, C.byref(st)), "stats")
        res[v].append((st.fwd_ms / max(1, st.fwd_launches), st.jac_ms / max(1, st.jac_launches), dt * 1e3,
                       2 * bench.FWD_MAC * st.fwd_points / (st.fwd_ms * 1e-3) / 1e12))
        sig = np.array([list(outs[i].t_cam_obj) + list(outs[i].code) + [outs[i].loss] for i in range(a.objects)], np.float32)
        if v not in ref: ref[v] = sig
        if r == 0 and v != a.variants[0]:
            same = np.array_equal(sig, ref[a.variants[0]])
            print(f"variant {v}: results identical to variant {a.variants[0]}: {same}", flush=True)
for v in a.variants:
    arr = np.array(res[v])
    print(f"V{v}: fwd ms/launch median {np.median(arr[:,0]):.2f} min {arr[:,0].min():.2f} | jac {np.median(arr[:,1]):.2f} | "
          f"batch ms {np.median(arr[:,2]):.1f} | fwd TF {np.median(arr[:,3]):.1f}", flush=True)
