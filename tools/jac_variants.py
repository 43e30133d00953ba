"""A/B the Jacobian kernel variants (DSR_JAC_VARIANT 0 = fp32, 8/12 = split-fp16) in one process."""
import ctypes as C, os, sys, time
import numpy as np
sys.path.insert(0, "dsp-slam-rgbd_amd"); sys.path.insert(0, ".")
import synthetic as S
from deep_sdf.workspace import decoder_from_state
from reconstruct import _libdsr as L
import bench
variants = [int(v) for v in sys.argv[1:]] or [0, 8, 12]
dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
batch, keep = bench.make_batch(dec, L.optim_params(S.KITTI_OPTIM), 64, 1000)
lib, ctx = dec.ctx.lib, dec.ctx
outs = (L.ObjectOut * 64)()
res = {v: [] for v in variants}
for r in range(2):
    for v in variants:
        os.environ["DSR_JAC_VARIANT"] = str(v)
        t0 = time.perf_counter()
        ctx.check(lib.dsr_batch_run(batch), "run"); ctx.check(lib.dsr_batch_download(batch, outs), "dl")
        dt = time.perf_counter() - t0
        st = L.Stats(); ctx.check(lib.dsr_batch_stats(batch, C.byref(st)), "stats")
        jtf = 2 * (bench.FWD_MAC + bench.BWD_MAC) * st.jac_points / (st.jac_ms * 1e-3) / 1e12
        res[v].append((st.fwd_ms / st.fwd_launches, st.jac_ms / st.jac_launches, dt * 1e3, jtf,
                       sum(outs[i].is_good for i in range(64))))
for v in variants:
    a = np.array(res[v])
    print(f"JV{v}: fwd {np.median(a[:,0]):.2f} ms | jac {np.median(a[:,1]):.2f} ms ({np.median(a[:,3]):.1f} TF) | batch {np.median(a[:,2]):.1f} ms | good {a[0,4]:.0f}/64")
