"""Marching cubes (MeshExtractor, optimizer.py:216-233 / utils.py:119-140) on the CPU.

The reference's mesher is skimage.measure.marching_cubes_lewiner (absent here, no meshes in
the reference): parity of vertex/face order is UNPINNED.  These tests pin the build's case
tables and the oracle restatement (oracle/dsr_mc.py) by the properties any correct
marching-cubes surface of a closed level set has, on analytic volumes.
"""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "tools"))


def _grid(d):
    g = (-1.0 + np.arange(d) * (2.0 / (d - 1))).astype(np.float32)
    return np.meshgrid(g, g, g, indexing="ij")


def _topology(v, f):
    e = np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]])
    und, cnt = np.unique(np.sort(e, 1), axis=0, return_counts=True)
    directed_unique = np.unique(e, axis=0).shape[0] == e.shape[0]
    chi = v.shape[0] - und.shape[0] + f.shape[0]
    return set(cnt.tolist()), directed_unique, chi


def test_tables_generated_file_is_current():
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "gen_mc_tables.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_tables_use_exactly_the_crossing_edges():
    from gen_mc_tables import build, edge_corners

    counts, tris = build()
    assert counts[0] == 0 and counts[255] == 0 and max(counts) <= 5
    for case in range(256):
        crossing = {e for e in range(12)
                    if ((case >> edge_corners(e)[0]) & 1) != ((case >> edge_corners(e)[1]) & 1)}
        used = {e for t in tris[case] for e in t}
        assert used == crossing, case


@pytest.mark.parametrize("d", [16, 33, 64])
def test_sphere_closed_outward_on_level_set(d):
    from oracle.dsr_mc import marching_cubes

    X, Y, Z = _grid(d)
    vol = (np.sqrt(X * X + Y * Y + Z * Z) - 0.6).astype(np.float32)
    v, f = marching_cubes(vol)
    uses, directed_unique, chi = _topology(v, f)
    assert uses == {2} and directed_unique and chi == 2
    n = np.cross(v[f[:, 1]] - v[f[:, 0]], v[f[:, 2]] - v[f[:, 0]])
    assert np.all(np.einsum("ij,ij->i", n, v[f].mean(1)) > 0)          # inside -> outside
    h = 2.0 / (d - 1)
    assert np.abs(np.linalg.norm(v, axis=1) - 0.6).max() < 0.05 * h     # linear interpolation
    area = 0.5 * np.linalg.norm(n, axis=1).sum()
    assert abs(area / (4 * np.pi * 0.36) - 1) < 0.02


def test_torus_genus_one():
    from oracle.dsr_mc import marching_cubes

    X, Y, Z = _grid(48)
    vol = (np.sqrt((np.sqrt(X * X + Y * Y) - 0.5) ** 2 + Z * Z) - 0.2).astype(np.float32)
    v, f = marching_cubes(vol)
    uses, directed_unique, chi = _topology(v, f)
    assert uses == {2} and directed_unique and chi == 0


def test_random_field_closed_and_oriented():
    """Ambiguous faces and cells everywhere: still every edge in exactly two faces, each
    direction once (neighbouring cells agree on every shared face)."""
    from oracle.dsr_mc import marching_cubes

    rng = np.random.default_rng(0)
    vol = rng.standard_normal((24, 24, 24)).astype(np.float32)
    vol[0], vol[-1], vol[:, 0], vol[:, -1], vol[:, :, 0], vol[:, :, -1] = (1.0,) * 6
    v, f = marching_cubes(vol)
    uses, directed_unique, _ = _topology(v, f)
    assert uses == {2} and directed_unique
    assert len(np.unique(f)) == v.shape[0]                              # no orphan vertices
