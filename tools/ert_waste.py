"""How much does the early-ray-termination schedule over-decode?  Along a reference
trajectory (tests/golden/f4_traj_<name>.npz: the reference's own per-iteration poses, codes
and depth samples) the fp32 oracle decodes every in-ball sample; a ray terminates at its first
in-ball rank with sdf <= -th (dsr_kernels.hpp: k_sample_pass).  Printed per iteration, as
fractions of the in-ball samples: the minimum any exact scheme must decode (through the
terminating sample), the default static pass schedule (dsr_api.hip: render_passes,
"8,12,16,20,24,32"), and a per-ray first window predicted from the previous iteration's
terminating rank followed by windows of w ranks.

Usage: python tools/ert_waste.py kitti0      (CPU, ~1 min)
"""
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)

import synthetic as S  # noqa: E402
from deep_sdf.workspace import fold_state  # noqa: E402
from oracle import dsr_oracle as O  # noqa: E402

def main():
    name = sys.argv[1]
    f = np.load(os.path.join(REPO, 'tests', 'golden', f'f4_traj_{name}.npz'))
    dec = O.Decoder(fold_state(S.make_decoder(1234), S.DEFAULT_SPECS))
    rays = f['obj_rays']; th = 0.01
    sched = [0,8,12,16,20,24,32]
    prev_t = None
    for i in range(int(f['n_iters_run'])):
        T = f['it_t_obj_cam'][i]; d = f['it_depths'][i]; z = f['it_z'][i]
        x = O.transform_points((rays[:, None, :] * d[:, None]).reshape(-1,3), T).reshape(rays.shape[0], 50, 3)
        inb = np.linalg.norm(x, axis=-1) < 1
        nin = inb.sum(1)
        sdf = np.full(inb.shape, np.nan, np.float32)
        xs = x[inb]
        sdf[inb] = O.decode_sdf(dec, z, xs.astype(np.float32)).reshape(-1)
        # rank-ordered sdf per ray
        tr = np.full(rays.shape[0], 10**6)
        for r in range(rays.shape[0]):
            v = sdf[r][inb[r]]
            k = np.nonzero(v <= -th)[0]
            if k.size: tr[r] = k[0]
        need = np.minimum(nin, tr + 1)
        # static schedule: passes end at boundaries; decode through end of pass containing t
        bnd = np.array(sched[1:] + [10**6])
        end = np.array([bnd[np.searchsorted(bnd, t, side='right')] if t < 10**6 else 10**6 for t in tr])
        stat = np.minimum(nin, end)
        # prediction: first pass [0, t_prev+1), then windows of w
        out = {}
        if prev_t is not None:
            for w in (1, 2, 4):
                p0 = np.minimum(prev_t + 1, 10**6)
                dec_n = np.where(tr < p0, np.minimum(nin, p0), 0)
                # rays alive after first window: decode windows of w until termination
                later = tr >= p0
                e2 = p0 + np.ceil((tr + 1 - p0) / w).astype(np.int64) * w
                dec_n = np.where(later, np.minimum(nin, np.where(tr < 10**6, e2, 10**6)), dec_n)
                dec_n = np.minimum(nin, dec_n)
                out[w] = dec_n.sum()
        print(f"it {i}: in-ball {nin.sum()} need {need.sum()} ({need.sum()/nin.sum():.3f}) static {stat.sum()} ({stat.sum()/nin.sum():.3f}) "
              + " ".join(f"pred w{w} {v} ({v/nin.sum():.3f})" for w, v in out.items())
              + f" term rays {np.sum(tr<10**6)} same-t as prev {np.sum(tr==prev_t) if prev_t is not None else -1}", flush=True)
        prev_t = tr


if __name__ == "__main__":
    main()
