"""where do the chunked first-pass scan's run-to-run decode counts come from?

GPU box, diagnostic build (`make -C dsp-slam-rgbd_amd/csrc exp_PROV.so`; the provenance arrays of
dsr_dev.hpp: PROV_IT).  Runs refine_sig.py's 8-object KITTI batch REPS times under the setting
that varied in round 5 (DSR_PRESCAN=1, DSR_STREAMS=4, lite kernel 1496) and compares every run
with the first: per (iteration, pass, ray) whether k_sample_pass found the ray alive, per
(iteration, sample) the lite value, per (iteration, ray) the depth index that terminated it.

Usage: DSR_LIB=$PWD/dsp-slam-rgbd_amd/csrc/exp_PROV.so DSR_TEST_HOOKS=1 DSR_PRESCAN=1 \\
       DSR_STREAMS=4 REPS=16 python tools/prov_diff.py
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)

import bench  # noqa: E402
import synthetic as S  # noqa: E402
from deep_sdf.workspace import decoder_from_state  # noqa: E402
from reconstruct import _libdsr as L  # noqa: E402

PROV_IT = 12
dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
lib, ctx = dec.ctx.lib, dec.ctx
lib.dsr_exp_prov.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 12
os.environ["DSR_LITE"] = "1"
REPS = int(os.environ.get("REPS", "16"))
M = 50


def one_run():
    h, keep = bench.make_batch(dec, L.optim_params(S.KITTI_OPTIM), 8, 1000)
    outs = (L.ObjectOut * 8)()
    ctx.check(lib.dsr_batch_run(h), "run")
    ctx.check(lib.dsr_batch_download(h, outs), "download")
    st = L.Stats()
    ctx.check(lib.dsr_batch_stats(h, ctypes.byref(st)), "stats")
    R, C = ctypes.c_int(), ctypes.c_int()
    ctx.check(lib.dsr_exp_prov(h, None, None, None, None, ctypes.byref(R), ctypes.byref(C), None, None,
                               None, None, None, None), "prov sizes")
    alive = np.zeros((PROV_IT, 64, R.value), np.int32)
    y = np.zeros((PROV_IT, C.value), np.float32)
    dset = np.zeros((PROV_IT, R.value), np.int32)
    xcc = np.zeros((PROV_IT, R.value, 2), np.int32)
    jf = np.zeros((PROV_IT, 64, R.value), np.int32)
    tt = np.zeros((PROV_IT, 65, R.value), np.uint32)
    hs = np.zeros((2, PROV_IT, R.value, 3), np.uint32)
    ri = np.zeros((2, PROV_IT, R.value, 2), np.uint32)
    nrm = np.zeros((PROV_IT, R.value, 12), np.float32)
    nrm2 = np.zeros((PROV_IT, R.value, 8), np.float32)
    ctx.check(lib.dsr_exp_prov(h, alive.ctypes.data, y.ctypes.data, dset.ctypes.data, xcc.ctypes.data, None, None,
                               jf.ctypes.data, tt.ctypes.data, hs.ctypes.data, ri.ctypes.data, nrm.ctypes.data,
                               nrm2.ctypes.data), "prov")
    inl2 = np.argwhere((nrm2[:, :, 0:4].view(np.uint32) != nrm2[:, :, 4:8].view(np.uint32)).any(-1))
    print(f"  k_sample_pass (first pass) rays whose in-loop |x| of samples 0..3 differ from the recomputed values: "
          f"{len(inl2)} of {int((nrm2[:, :, 4] != 0).sum())}", flush=True)
    inl = np.argwhere((nrm[:, :, 0:4].view(np.uint32) != nrm[:, :, 4:8].view(np.uint32)).any(-1))
    print(f"  scan rays whose in-loop |x| of samples 0..3 differ from the same values recomputed after the loop: "
          f"{len(inl)}" + "".join(f"\n    it {a} ray {b}: loop {nrm[a, b, 0:4].tolist()} after {nrm[a, b, 4:8].tolist()} "
                                   f"depths {nrm[a, b, 8:12].tolist()}" for a, b in inl[:6]), flush=True)
    # rinfo: the value the first k_sample_pass read vs the value k_sample_scan wrote, and when
    vis = (ri[0, :, :, 1] != 0) & (ri[1, :, :, 1] != 0)
    bad = np.argwhere(vis & (ri[0, :, :, 0] != ri[1, :, :, 0]))
    dt = ri[1, :, :, 1].astype(np.int64) - ri[0, :, :, 1].astype(np.int64)
    print(f"  rinfo reads of the first pass that differ from the scan's write: {len(bad)} of {int(vis.sum())}; "
          f"read - write time over all rays: min {int(dt[vis].min()) if vis.any() else 0} ticks"
          + "".join(f"\n    it {a} ray {b}: scan wrote {int(ri[0, a, b, 0]):#x}, pass read {int(ri[1, a, b, 0]):#x}, "
                    f"read - write {int(dt[a, b])} ticks" for a, b in bad[:8]), flush=True)
    # state seen by the chunked scan vs the state k_iter_begin wrote (object key = its first ray)
    obj_keys = np.nonzero(hs[0, 0, :, 1])[0]
    stale = []
    for it in range(PROV_IT):
        for c in np.nonzero(hs[1, it, :, 1])[0]:
            o = obj_keys[np.searchsorted(obj_keys, c, side="right") - 1]
            if hs[1, it, c, 0] != hs[0, it, o, 0]:
                stale.append((it, int(o), int(c), int(hs[1, it, c, 1]) - int(hs[0, it, o, 1]),
                              int(hs[0, it, o, 2]), int(hs[1, it, c, 2])))
    print(f"  scan chunks that staged a pose / depth set other than k_iter_begin's: {len(stale)}"
          + "".join(f"\n    it {a} object@{b} chunk@{c}: scan read - k_iter_begin write {d} ticks, XCC writer {e} "
                    f"reader {g}" for a, b, c, d, e, g in stale[:8]), flush=True)
    rx = np.where(alive == 0, -1, (alive + 1) // 1024)          # the reading workgroup's XCC
    alive = np.where(alive == 0, 0, alive - 1024 * rx)
    rec = np.array([list(o.t_cam_obj) + list(o.code) + [o.loss] for o in outs], np.float32)
    lib.dsr_batch_destroy(h)
    return st.fwd_points, st.refine_points, rec, alive, y, dset, xcc, rx, jf, tt, hs, ri, nrm


runs = [one_run() for _ in range(REPS)]
f0, r0, rec0, a0, y0, s0, x0, rx0, jf0, t0, hs0, ri0, nrm0 = runs[0]
print(f"run 0: fwd {f0} refine {r0}", flush=True)
stat = {"same_xcd": 0, "other_xcd": 0}
for i, (f, r, rec, a, y, s, x, rx, jf, tt, hs, ri, nrm) in enumerate(runs[1:], 1):
    dh = np.argwhere(hs[0, :, :, 0] != hs0[0, :, :, 0])
    dr = np.argwhere(ri[0, :, :, 0] != ri0[0, :, :, 0])
    print(f"  vs run 0: k_iter_begin pose/depth checksums differing {len(dh)} (first {dh[:3].tolist()}); scan rinfo "
          f"writes differing {len(dr)}" + "".join(f"\n    it {a} ray {b}: rinfo {int(ri0[0, a, b, 0]):#x} vs "
                                               f"{int(ri[0, a, b, 0]):#x}; |x| 0..3 run0 loop {nrm0[a, b, 0:4].tolist()} "
                                               f"after {nrm0[a, b, 4:8].tolist()} run{i} loop {nrm[a, b, 0:4].tolist()} "
                                               f"after {nrm[a, b, 4:8].tolist()} depths {nrm[a, b, 8:12].tolist()}"
                                               for a, b in dr[:4]), flush=True)
    same_rec = np.array_equal(rec.view(np.uint32), rec0.view(np.uint32))
    both = ~np.isnan(y) & ~np.isnan(y0)
    vdiff = both & (y.view(np.uint32) != y0.view(np.uint32))
    only = np.isnan(y) != np.isnan(y0)
    adiff = np.argwhere(a != a0)
    sdiff = np.argwhere(s != s0)
    print(f"run {i}: fwd {f} ({f - f0:+d}) refine {r} ({r - r0:+d}) records {'equal' if same_rec else 'DIFFER'}; "
          f"lite values differing on commonly decoded samples {int(vdiff.sum())}; samples decoded in one run only "
          f"{int(only.sum())}; (it, pass, ray) alive/emit entries differing {len(adiff)}; dead-setter entries "
          f"differing {len(sdiff)}", flush=True)
    for it, ra, ray in adiff[:12]:
        j0, j1 = int(s0[it, ray]), int(s[it, ray])
        print(f"   it {it} pass@{ra} ray {ray}: run0 {a0[it, ra, ray]} run{i} {a[it, ra, ray]}; terminated by j "
              f"run0 {j0 if j0 < 2**30 else '-'} run{i} {j1 if j1 < 2**30 else '-'}; XCC clear / set / read "
              f"run0 {x0[it, ray, 0]} / {x0[it, ray, 1]} / {rx0[it, ra, ray]} run{i} {x[it, ray, 0]} / {x[it, ray, 1]} / "
              f"{rx[it, ra, ray]}", flush=True)
        stat["same_xcd" if x[it, ray, 0] == rx[it, ra, ray] else "other_xcd"] += 1
        for pra in range(ra + 1):
            if a0[it, pra, ray] != 0 or a[it, pra, ray] != 0:
                print(f"      pass@{pra}: emitted run0 {a0[it, pra, ray] - 1} from j {jf0[it, pra, ray]} (t {t0[it, pra, ray]}) "
                      f"run{i} {a[it, pra, ray] - 1} from j {jf[it, pra, ray]} (t {tt[it, pra, ray]})")
        print(f"      first set of the flag: run0 t {t0[it, 64, ray]} run{i} t {tt[it, 64, ray]}; read of pass@{ra} "
              f"minus set: run0 {int(t0[it, ra, ray]) - int(t0[it, 64, ray])} run{i} "
              f"{int(tt[it, ra, ray]) - int(tt[it, 64, ray])} (10 ns ticks)")
    if vdiff.any():
        it, smp = np.argwhere(vdiff)[0]
        print(f"   first differing lite value: it {it} sample {smp}: {y0[it, smp]!r} vs {y[it, smp]!r}")
    for it, ray in sdiff[:6]:
        print(f"   dead setter it {it} ray {ray}: run0 {s0[it, ray]} run{i} {s[it, ray]}")

# over every run: how often the clearing and the reading workgroup share an XCD at all (for the
# rays a dead flag was set on), against the differing entries above
tot = {"same": 0, "all": 0}
for (f, r, rec, a, y, s, x, rx, jf, tt, hs, ri, nrm) in runs:
    for it in range(PROV_IT):
        rays = np.nonzero(s[it] < 2**30)[0]
        for ra in np.unique(np.nonzero(a[it] != 0)[0]):
            if ra == 0:
                continue
            rr = rays[a[it, ra, rays] != 0]
            tot["same"] += int((x[it, rr, 0] == rx[it, ra, rr]).sum())
            tot["all"] += len(rr)
print(f"differing reads: clearer's XCC == reader's XCC {stat['same_xcd']}, other {stat['other_xcd']}; over all "
      f"reads of terminated rays in later passes: same XCC {tot['same']} of {tot['all']}")
