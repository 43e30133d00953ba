"""The CPU oracle (numpy fp32) from the 256 ulp-perturbed starts of golden F13 (kitti0, kitti5), per
iteration (K, loss), against the reference's own F13 clouds — a third fp32 implementation of
the algorithm, to size how far two correct fp32 implementations' per-iteration clouds sit apart
(tests/test_gpu_contract.py::test_ens256_distribution_per_iteration).  CPU only:

    python tools/oracle_ens256.py [jobs] [name]    -> tests/golden/f16_oracle_ens256_<name>.npz
    DSR_ORACLE_FP64=1 DSR_ENS_MEMBERS=64 python tools/oracle_ens256.py [jobs] [name]
                                                   -> tests/golden/f19_oracle64_ens64_<name>.npz

The second form runs the oracle in fp64 from the first 64 of the same starts: each member's
exact-arithmetic trajectory (to ~1e-16), the reference the per-iteration clouds of the fp32
implementations (the reference, the GPU, the fp32 oracle) are measured against.

The output is the oracle's, not the reference's: it is test data for the GPU test's yardstick.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import synthetic as S  # noqa: E402

_W = {}
FP64 = os.environ.get("DSR_ORACLE_FP64", "0") == "1"
MEMBERS = int(os.environ.get("DSR_ENS_MEMBERS", "256"))


def _init(name):
    from deep_sdf.workspace import fold_state
    from oracle import dsr_oracle as O
    from threadpoolctl import threadpool_limits

    threadpool_limits(1)
    g = os.path.join(REPO, "tests", "golden")
    _W.update(O=O, f=dict(np.load(os.path.join(g, f"f4_traj_{name}.npz"), allow_pickle=False)),
              e=dict(np.load(os.path.join(g, f"f13_ens256_{name}.npz"), allow_pickle=False)),
              dec=O.Decoder(fold_state(S.make_decoder(1234), S.DEFAULT_SPECS), dtype=np.float64 if FP64 else np.float32),
              P=O.OptimParams.from_cfg(S.KITTI_OPTIM))


def _member(m):
    f, O = _W["f"], _W["O"]
    r = O.reconstruct_object(_W["dec"], _W["P"], _W["e"]["t_init"][m], f["obj_pts"], f["obj_rays"], f["obj_depth"])
    n = len(r.trace)
    k = np.full(10, -1, np.int32)
    ls = np.full(10, np.nan)
    lr = np.full(10, np.nan)
    for i, t in enumerate(r.trace[:10]):
        k[i], ls[i], lr[i] = t.k, t.sdf_loss, t.render_loss
    return np.asarray(r.t_cam_obj, np.float32), np.asarray(r.code, np.float32), float(r.loss), bool(r.is_good), k, ls, lr, n


def _indexed(m):
    return m, _member(m)


def main():
    jobs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    name = sys.argv[2] if len(sys.argv) > 2 else "kitti0"
    tag = f"oracle64_ens{MEMBERS}" if FP64 else f"oracle_ens{MEMBERS}"
    part = f"/tmp/{tag}_{name}_partial.npy"
    done = {}
    if os.path.exists(part):                 # resume a run that was cut off
        done = np.load(part, allow_pickle=True).item()
    todo = [m for m in range(MEMBERS) if m not in done]
    with mp.get_context("fork").Pool(jobs, initializer=_init, initargs=(name,)) as pool:
        for m, r in pool.imap_unordered(_indexed, todo, chunksize=1):
            done[m] = r
            np.save(part, np.array(done, dtype=object), allow_pickle=True)
            print(f"member {m} done ({len(done)}/{MEMBERS})", flush=True)
    res = [done[m] for m in range(MEMBERS)]
    out = dict(t_cam_obj=np.stack([r[0] for r in res]), code=np.stack([r[1] for r in res]),
               loss=np.array([r[2] for r in res]), is_good=np.array([r[3] for r in res]),
               it_k=np.stack([r[4] for r in res]), it_sdf_loss=np.stack([r[5] for r in res]),
               it_render_loss=np.stack([r[6] for r in res]), n_trace=np.array([r[7] for r in res]))
    fn = f"f19_{tag}_{name}.npz" if FP64 else f"f16_{tag}_{name}.npz"
    np.savez_compressed(os.path.join(REPO, "tests", "golden", fn), **out)
    print("done", out["is_good"].all(), np.unique(out["n_trace"]))


if __name__ == "__main__":
    main()
