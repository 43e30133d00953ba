"""F9: the reference's mesh-extraction path up to triangulation (build container only).

    python tests/golden/make_mesher.py        # writes tests/golden/f9_mesher.npz

``MeshExtractor.extract_mesh_from_code`` (reference optimizer.py:216-233) is
create_voxel_grid (utils.py:97-116) -> decode_sdf over the grid (optimizer.py:225-226)
-> ``.view(d, d, d)`` -> ``convert_sdf_voxels_to_mesh`` (utils.py:119-140):
skimage's ``marching_cubes_lewiner`` with ``spacing = 2/(d-1)``, then the origin
shift of utils.py:133-138 and ``astype(float32)`` (optimizer.py:228).  skimage is
absent here (and the lewiner entry point is gone from modern skimage), so the
triangulation itself stays unpinned; everything around it is recorded from the
reference: the grid points, the decoded grid exactly as the reference hands it to
marching cubes (captured by a stand-in for ``measure.marching_cubes_lewiner`` that
also returns a known vertex set in skimage's output convention — index * spacing,
float64), and the vertices the reference makes of them.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "dsp-slam-rgbd_amd"))
sys.path.insert(0, HERE)

import synthetic as S  # noqa: E402
import refshim  # noqa: E402
import make_golden as MG  # noqa: E402

DIM = 32


def main():
    import torch

    torch.set_num_threads(1)
    ref = refshim.load()
    dec = refshim.build_decoder(S.make_decoder(MG.DECODER_SEED), S.DEFAULT_SPECS)
    rng = np.random.default_rng(909)
    code = (0.05 * rng.standard_normal(64)).astype(np.float32)
    grid = ref.utils.create_voxel_grid(vol_dim=DIM).numpy()
    spacing = 2.0 / (DIM - 1)
    idx = np.concatenate([rng.integers(0, DIM - 1, (200, 3)) + rng.uniform(0, 1, (200, 3)) * np.eye(3)[
        rng.integers(0, 3, 200)], np.array([[0, 0, 0], [DIM - 1, DIM - 1, DIM - 1], [0.5, 0, DIM - 1.5]])])
    seen = {}

    def lewiner_standin(volume, level=0.0, spacing=(1.0, 1.0, 1.0), **kw):
        seen["volume"] = np.array(volume, copy=True)
        seen["level"] = level
        seen["spacing"] = np.asarray(spacing, np.float64)
        verts = idx * np.asarray(spacing, np.float64)           # skimage: index * spacing
        return verts.copy(), np.zeros((0, 3), np.int64), np.zeros_like(verts), np.zeros(len(verts))

    ref.utils.measure.marching_cubes_lewiner = lewiner_standin
    mex = ref.optimizer.MeshExtractor(dec, 64, DIM)
    out = mex.extract_mesh_from_code(code.copy())
    np.savez_compressed(os.path.join(HERE, "f9_mesher.npz"), dim=np.array(DIM), code=code, grid=grid,
                        volume=seen["volume"], level=np.array(seen["level"]), spacing=seen["spacing"],
                        verts_index=idx, verts_out=np.asarray(out.vertices), verts_dtype=np.array(
                            str(np.asarray(out.vertices).dtype)), torch=np.array(torch.__version__))
    print("f9 written: grid", grid.shape, "volume", seen["volume"].shape, "verts", out.vertices.shape)


if __name__ == "__main__":
    main()
