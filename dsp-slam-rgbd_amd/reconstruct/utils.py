"""``reconstruct/utils.py`` of the reference, every public name (utils.py:26-161).

Same names and behaviour the C++ side relies on (src/System.cc:95-98):
``get_configs(path)`` returns an attribute dict that raises ``KeyError`` on a
missing key (``ForceKeyErrorDict``, utils.py:82-90), ``get_decoder(cfg)`` returns
the decoder handle built from ``cfg.DeepSDF_DIR`` (utils.py:93-94).  The mesher half
(``create_voxel_grid``, ``convert_sdf_voxels_to_mesh``, ``write_mesh_to_ply``) and the
viewer helpers the reference's scripts import (``color_table``, ``set_view``:
reconstruct_frame.py:20, visualize_map.py:22) keep their names too.
"""
from __future__ import annotations

import json

import numpy as np


# the reference's visualisation palette (utils.py:26-37), RGB in [0, 1]: red, green, blue,
# magenta, orange, purple, cyan, lime, pink, teal
color_table = [[r / 255., g / 255., b / 255.] for r, g, b in (
    (230, 0, 0), (60, 180, 75), (0, 0, 255), (255, 0, 255), (255, 165, 0),
    (128, 0, 128), (0, 255, 255), (210, 245, 60), (250, 190, 190), (0, 128, 128))]


def set_view(vis, dist=100., theta=np.pi / 6.):
    """utils.py:40-55: point an Open3D visualiser's camera at the world origin from `dist`
    along its z axis, tilted by `theta` about x (world -> eye extrinsic).  Needs only the
    visualiser object the caller passes (no open3d import here)."""
    ctl = vis.get_view_control()
    cam = ctl.convert_to_pinhole_camera_parameters()
    c, s = np.cos(theta), np.sin(theta)
    cam.extrinsic = np.array([[1., 0., 0., 0.],
                              [0., c, -s, 0.],
                              [0., s, c, dist],
                              [0., 0., 0., 1.]])
    ctl.convert_from_pinhole_camera_parameters(cam)


class ForceKeyErrorDict(dict):
    """addict.Dict-like attribute dict whose missing keys raise KeyError (utils.py:82-84)."""

    def __init__(self, *args, **kwargs):
        super().__init__()
        for k, v in dict(*args, **kwargs).items():
            self[k] = self._conv(v)

    @classmethod
    def _conv(cls, v):
        if isinstance(v, dict) and not isinstance(v, ForceKeyErrorDict):
            return cls(v)
        if isinstance(v, list):
            return [cls._conv(x) for x in v]
        return v

    def __getattr__(self, k):
        if k.startswith("__") and k.endswith("__"):
            raise AttributeError(k)
        try:
            return self[k]
        except KeyError:
            raise KeyError(k) from None

    def __setattr__(self, k, v):
        self[k] = self._conv(v)

    def __missing__(self, key):
        raise KeyError(key)


def read_calib_file(filepath):
    """utils.py:58-73: a KITTI calibration file as {key: float64 array}; parsing stops at the
    first empty line and keys whose values are not all numbers (dates) are skipped.  Used by
    the reference's kitti_sequence.py (data ingest, kept by the C++ caller)."""
    data = {}
    with open(filepath, "r") as f:
        for line in f.readlines():
            if line == "\n":
                break
            key, value = line.split(":", 1)
            try:
                data[key] = np.array([float(x) for x in value.split()])
            except ValueError:
                pass
    return data


def load_velo_scan(file):
    """utils.py:76-79: a velodyne .bin scan as an (N, 4) float32 array (x, y, z, reflectance)."""
    return np.fromfile(file, dtype=np.float32).reshape((-1, 4))


def get_configs(cfg_file):
    """utils.py:87-90."""
    with open(cfg_file) as f:
        cfg_dict = json.load(f)
    return ForceKeyErrorDict(**cfg_dict)


def get_decoder(configs, device=None):
    """utils.py:93-94: ``config_decoder(configs.DeepSDF_DIR)`` -> device decoder handle."""
    from deep_sdf.workspace import config_decoder

    return config_decoder(configs.DeepSDF_DIR, device=device)


def create_voxel_grid(vol_dim=128):
    """utils.py:97-116.  Note the reference's ``LongTensor / vol_dim`` is TRUE division
    in torch >= 1.6 (fp32), so its x/y columns are not integer lattice indices; this
    restates that fp32 arithmetic exactly (verified against torch in the tests)."""
    voxel_origin = [-1, -1, -1]
    voxel_size = 2.0 / (vol_dim - 1)
    idx = np.arange(vol_dim ** 3, dtype=np.int64)
    fidx = idx.astype(np.float32)
    fv = np.float32(vol_dim)
    values = np.zeros((vol_dim ** 3, 3), np.float32)
    values[:, 2] = idx % vol_dim
    values[:, 1] = np.remainder(fidx / fv, fv)
    values[:, 0] = np.remainder((fidx / fv) / fv, fv)
    values[:, 0] = values[:, 0] * np.float32(voxel_size) + np.float32(voxel_origin[2])
    values[:, 1] = values[:, 1] * np.float32(voxel_size) + np.float32(voxel_origin[1])
    values[:, 2] = values[:, 2] * np.float32(voxel_size) + np.float32(voxel_origin[0])
    return values


def convert_sdf_voxels_to_mesh(pytorch_3d_sdf_tensor, level=0.0, device=None):
    """utils.py:119-140 on device (``dsr_mc_volume``): marching cubes of an (n, n, n) SDF
    volume (torch tensor or array, C order — the grid order of ``create_voxel_grid``), vertices
    as voxel index x 2/(n-1) - 1 (the reference's spacing and origin shift), faces as vertex
    indices.  Returns (vertices float32 (V, 3), faces int32 (F, 3)) — float32 because the
    build's only caller, ``MeshExtractor``, casts to it anyway (optimizer.py:228).  The
    triangulation is the build's marching cubes, not skimage's ``marching_cubes_lewiner``
    (absent here: parity unpinned)."""
    import ctypes as C

    from reconstruct import _libdsr as L

    t = pytorch_3d_sdf_tensor
    if hasattr(t, "detach"):
        t = t.detach().cpu().numpy()
    vol = np.ascontiguousarray(t, dtype=np.float32)
    if vol.ndim != 3 or len(set(vol.shape)) != 1:
        raise ValueError(f"expected an (n, n, n) volume, got shape {vol.shape}")
    d = vol.shape[0]
    ctx = L.Context.get(device)
    verts = np.zeros((3 * d ** 3, 3), np.float32)
    faces = np.zeros((5 * (d - 1) ** 3, 3), np.int32)
    nv, nf = C.c_int(), C.c_int()
    ctx.check(ctx.lib.dsr_mc_volume(ctx.handle, L.fptr(vol), d, float(level), L.fptr(verts), verts.shape[0],
                                    L.iptr(faces), faces.shape[0], C.byref(nv), C.byref(nf)), "dsr_mc_volume")
    return verts[:nv.value].copy(), faces[:nf.value].copy()


# PLY layout plyfile.PlyData([vertex(x,y,z f4), face(vertex_indices i4 x3)]).write() produces
# (utils.py:143-161): binary, native (little-endian) byte order, list counts as uchar.
_PLY_HEADER = ("ply\nformat binary_little_endian 1.0\nelement vertex {nv}\nproperty float x\n"
               "property float y\nproperty float z\nelement face {nf}\n"
               "property list uchar int vertex_indices\nend_header\n")


def write_mesh_to_ply(v, f, ply_filename_out):
    """utils.py:141-161 without plyfile: the same binary PLY."""
    v = np.ascontiguousarray(v, dtype="<f4").reshape(-1, 3)
    f = np.ascontiguousarray(f, dtype="<i4").reshape(-1, 3)
    rec = np.zeros(f.shape[0], dtype=[("n", "u1"), ("idx", "<i4", (3,))])
    rec["n"] = 3
    rec["idx"] = f
    with open(ply_filename_out, "wb") as fh:
        fh.write(_PLY_HEADER.format(nv=v.shape[0], nf=f.shape[0]).encode("ascii"))
        fh.write(v.tobytes())
        fh.write(rec.tobytes())


def read_mesh_ply(path):
    """Inverse of write_mesh_to_ply (triangle meshes in that layout only)."""
    with open(path, "rb") as fh:
        data = fh.read()
    end = data.index(b"end_header\n") + len(b"end_header\n")
    head = data[:end].decode("ascii").split("\n")
    nv = int(next(x for x in head if x.startswith("element vertex")).split()[-1])
    nf = int(next(x for x in head if x.startswith("element face")).split()[-1])
    v = np.frombuffer(data, dtype="<f4", count=3 * nv, offset=end).reshape(nv, 3)
    rec = np.frombuffer(data, dtype=[("n", "u1"), ("idx", "<i4", (3,))], count=nf, offset=end + 12 * nv)
    if nf and not np.all(rec["n"] == 3):
        raise ValueError("not a triangle mesh")
    return v.copy(), rec["idx"].copy()
