"""CPU restatement of libdsr's marching cubes (test infrastructure only).

Parity UNPINNED against the reference: reconstruct/utils.py:119-140 calls
skimage.measure.marching_cubes_lewiner (scikit-image <= 0.18, not installable here) and
the reference holds no meshes.  This module restates the BUILD's algorithm (case tables
from tools/gen_mc_tables.py, edge-owned vertices, scan-ordered output) so the GPU kernels
are checked bit-for-bit against it, while tests/test_mesh_*.py check the mesh itself by
properties the reference's output also has (vertices on the level set, closed and
consistently oriented surfaces, Euler characteristic, area/volume of analytic shapes).
The vertex transform follows utils.py:131-138 (index * spacing, then + origin -1).
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools"))
from gen_mc_tables import build as _build_tables, edge_corners  # noqa: E402

_COUNTS, _TRIS = _build_tables()


def vertex_transform(pos, d):
    """Grid-index positions (V, 3) float64 -> vertices: skimage's ``index * spacing``
    (spacing 2/(d-1) in float64), the reference's origin shift (utils.py:131-138) in
    float64, then ``astype(float32)`` (optimizer.py:228).  Pinned by golden F9."""
    spacing = 2.0 / (d - 1)                                     # utils.py:127 (float64)
    return (-1.0 + np.asarray(pos, np.float64) * spacing).astype(np.float32)


def marching_cubes(vol, level=0.0):
    """vol: (d, d, d) float32 indexed [i][j][k] = value at grid point (x_i, y_j, z_k).
    Returns vertices (V, 3) float32 in [-1, 1]^3 and faces (F, 3) int32, ordered like the
    device kernels: vertices by (grid point, axis) of the owning edge, faces by cell and
    table order."""
    vol = np.asarray(vol, np.float32)
    d = vol.shape[0]
    f32 = np.float32
    spacing = 2.0 / (d - 1)                                     # utils.py:127 (float64)
    lev = f32(level)
    inside = vol < lev
    # edge crossings owned by grid points: axis 0 (i), 1 (j), 2 (k)
    cross = np.zeros((d, d, d, 3), bool)
    cross[:-1, :, :, 0] = inside[:-1] != inside[1:]
    cross[:, :-1, :, 1] = inside[:, :-1] != inside[:, 1:]
    cross[:, :, :-1, 2] = inside[:, :, :-1] != inside[:, :, 1:]
    flat = cross.reshape(-1)
    vidx = np.cumsum(flat) - 1
    nv = int(flat.sum())
    verts = np.zeros((nv, 3), np.float32)
    ids = np.nonzero(flat)[0]
    pt, ax = ids // 3, ids % 3
    i, j, k = pt // (d * d), (pt // d) % d, pt % d
    step = np.stack([ax == 0, ax == 1, ax == 2], 1).astype(np.int64)
    v0 = vol[i, j, k].astype(np.float64)
    v1 = vol[i + step[:, 0], j + step[:, 1], k + step[:, 2]].astype(np.float64)
    t = (np.float64(lev) - v0) / (v1 - v0)                      # fp64 like skimage's Cython
    base = np.stack([i, j, k], 1).astype(np.float64)
    pos = base + step * t[:, None]
    verts[:] = vertex_transform(pos, d)                           # utils.py:128-138, optimizer.py:228
    # cells
    c = np.arange((d - 1) ** 3)
    ci, cj, ck = c // ((d - 1) ** 2), (c // (d - 1)) % (d - 1), c % (d - 1)
    case = np.zeros(c.shape[0], np.int64)
    for corner in range(8):
        case |= inside[ci + (corner & 1), cj + ((corner >> 1) & 1), ck + ((corner >> 2) & 1)].astype(
            np.int64) << corner
    faces = []
    counts = np.array(_COUNTS)[case]
    for cell in np.nonzero(counts)[0]:
        for tri in _TRIS[case[cell]]:
            f = []
            for e in tri:
                c0, _ = edge_corners(e)
                a = e // 4
                gi, gj, gk = ci[cell] + (c0 & 1), cj[cell] + ((c0 >> 1) & 1), ck[cell] + ((c0 >> 2) & 1)
                f.append(vidx[((gi * d + gj) * d + gk) * 3 + a])
            faces.append(f)
    return verts, np.asarray(faces, np.int32).reshape(-1, 3)
