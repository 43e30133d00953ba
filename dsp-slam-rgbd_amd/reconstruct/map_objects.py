"""MapObjects.txt — the on-disk interchange of reconstructed objects.

Writer side: System::SaveMapObjects (src/System_util.cc:123-145) — per object, in id order:
  line 1  mnId
  line 2  the 3x4 Sim(3) T_wo, row-major, `std::fixed << setprecision(9)`, space-separated
  line 3  the shape code as an Eigen row vector (`<< code.transpose()`): fixed, 9 decimals,
          every coefficient right-aligned to the widest one, single-space separated.
Reader side: extract_map_objects.py:46-63 — id, pose (+ [0,0,0,1] row) saved as
objects/<id>.npy, code -> MeshExtractor -> objects/<id>.ply.
"""
from __future__ import annotations

import os

import numpy as np

from reconstruct.utils import write_mesh_to_ply


def _fixed9(x):
    return f"{float(x):.9f}"


def format_map_objects(objects):
    """objects: iterable of (id, T_wo (3x4 or 4x4), code (L,)) -> MapObjects.txt text."""
    out = []
    for oid, T, code in sorted(objects, key=lambda o: int(o[0])):
        T = np.asarray(T, np.float32)[:3, :4]
        out.append(str(int(oid)))
        out.append(" ".join(_fixed9(x) for x in T.reshape(-1)))
        cs = [_fixed9(x) for x in np.asarray(code, np.float32).reshape(-1)]
        w = max((len(c) for c in cs), default=0)
        out.append(" ".join(c.rjust(w) for c in cs))
    return "".join(line + "\n" for line in out)


def write_map_objects(path, objects):
    with open(path, "w") as f:
        f.write(format_map_objects(objects))


def read_map_objects(path):
    """extract_map_objects.py:46-63: list of (id, pose 4x4 float64, code float32)."""
    with open(path) as f:
        lines = f.readlines()
    res = []
    for i in range(len(lines) // 3):
        oid = int(lines[3 * i])
        pose = np.asarray([float(x) for x in lines[3 * i + 1].strip().split(" ")]).reshape(3, 4)
        pose = np.concatenate([pose, np.array([0., 0., 0., 1.]).reshape(1, 4)], axis=0)
        code = [float(item) for item in lines[3 * i + 2].strip().split(" ") if len(item) > 0]
        res.append((oid, pose, np.asarray(code).astype(np.float32)))
    return res


def extract_map_objects(map_dir, mesh_extractor):
    """The body of extract_map_objects.py: objects/<id>.npy (pose) and objects/<id>.ply
    (mesh of the code through `mesh_extractor`, a reconstruct.optimizer.MeshExtractor)."""
    save_dir = os.path.join(map_dir, "objects")
    os.makedirs(save_dir, exist_ok=True)
    done = []
    for oid, pose, code in read_map_objects(os.path.join(map_dir, "MapObjects.txt")):
        np.save(os.path.join(save_dir, "%d.npy" % oid), pose)
        mesh = mesh_extractor.extract_mesh_from_code(code)
        write_mesh_to_ply(mesh.vertices, mesh.faces, os.path.join(save_dir, "%d.ply" % oid))
        done.append(oid)
    return done
