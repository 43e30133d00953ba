"""MapObjects.txt writer/reader (System_util.cc:123-145 <-> extract_map_objects.py:46-63) and
the binary PLY of write_mesh_to_ply (utils.py:141-161), on the CPU."""
from __future__ import annotations

import numpy as np


def _objects(n=3, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        T = np.eye(4, dtype=np.float32)
        T[:3, :3] = (rng.standard_normal((3, 3)) * 0.5).astype(np.float32)
        T[:3, 3] = rng.standard_normal(3).astype(np.float32) * 10
        out.append((7 * i + 3, T, rng.standard_normal(64).astype(np.float32)))
    return out[::-1]                                   # writer sorts by id (MapObject::lId)


def test_format_matches_cpp_stream_output():
    from reconstruct.map_objects import format_map_objects

    T = np.eye(4, dtype=np.float32)
    T[0, 3] = -1.5
    code = np.array([0.25, -1.0, 10.125], np.float32)
    lines = format_map_objects([(5, T, code)]).split("\n")
    assert lines[0] == "5"
    # std::fixed << setprecision(9), " " between coefficients, no trailing space
    assert lines[1] == ("1.000000000 0.000000000 0.000000000 -1.500000000 "
                        "0.000000000 1.000000000 0.000000000 0.000000000 "
                        "0.000000000 0.000000000 1.000000000 0.000000000")
    # Eigen row vector: coefficients right-aligned to the widest
    assert lines[2] == " 0.250000000 -1.000000000 10.125000000"


def test_round_trip(tmp_path):
    from reconstruct.map_objects import read_map_objects, write_map_objects

    objs = _objects()
    p = tmp_path / "MapObjects.txt"
    write_map_objects(str(p), objs)
    back = read_map_objects(str(p))
    assert [b[0] for b in back] == sorted(o[0] for o in objs)
    for (oid, pose, code), ref in zip(back, sorted(objs, key=lambda o: o[0])):
        assert pose.shape == (4, 4) and np.array_equal(pose[3], [0, 0, 0, 1])
        assert np.allclose(pose[:3], ref[1][:3], atol=5e-10 + 1e-9 * np.abs(ref[1][:3]).max())
        assert code.dtype == np.float32 and np.allclose(code, ref[2], atol=1e-9)


def test_ply_layout_and_round_trip(tmp_path):
    from reconstruct.utils import read_mesh_ply, write_mesh_to_ply

    v = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1]], np.float32)
    f = np.array([[0, 2, 1], [0, 1, 3], [0, 3, 2], [1, 2, 3]], np.int32)
    p = tmp_path / "m.ply"
    write_mesh_to_ply(v, f, str(p))
    raw = p.read_bytes()
    head = raw[:raw.index(b"end_header\n") + 11].decode()
    assert head.splitlines() == ["ply", "format binary_little_endian 1.0", "element vertex 4",
                                 "property float x", "property float y", "property float z",
                                 "element face 4", "property list uchar int vertex_indices",
                                 "end_header"]
    assert len(raw) == len(head) + 4 * 12 + 4 * 13
    v2, f2 = read_mesh_ply(str(p))
    assert np.array_equal(v, v2) and np.array_equal(f, f2)
