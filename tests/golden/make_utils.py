"""F11: the reference's viewer helpers in reconstruct/utils.py (build container only).

    python tests/golden/make_utils.py        # writes tests/golden/f11_utils.npz

``color_table`` (utils.py:26-37) and ``set_view`` (utils.py:40-55) are imported by the
reference's scripts (reconstruct_frame.py:20, visualize_map.py:22).  The palette is recorded
as the reference module holds it; ``set_view`` is run on a stand-in for the Open3D
visualiser (open3d is absent here) that records the extrinsic the function installs.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import refshim  # noqa: E402

VIEWS = [(100.0, np.pi / 6.0), (20.0, 0.0), (35.5, 0.3)]   # default, reconstruct_frame.py:84, other


class _Vis:
    """Open3D Visualizer stand-in: get_view_control() -> a control whose pinhole parameters
    carry an `extrinsic`; the installed one is kept."""

    def __init__(self):
        self.installed = None
        vis = self

        class _Ctl:
            def convert_to_pinhole_camera_parameters(self):
                return types.SimpleNamespace(extrinsic=np.zeros((4, 4)))

            def convert_from_pinhole_camera_parameters(self, cam):
                vis.installed = np.array(cam.extrinsic, dtype=np.float64)

        self._ctl = _Ctl()

    def get_view_control(self):
        return self._ctl


def main():
    ref = refshim.load()
    ext = []
    for dist, theta in VIEWS:
        v = _Vis()
        ref.utils.set_view(v, dist=dist, theta=theta)
        ext.append(v.installed)
    v = _Vis()
    ref.utils.set_view(v)
    ext.append(v.installed)                                     # the defaults
    np.savez_compressed(os.path.join(HERE, "f11_utils.npz"),
                        color_table=np.asarray(ref.utils.color_table, np.float64),
                        views=np.asarray(VIEWS, np.float64), extrinsics=np.stack(ext))
    print("f11 written:", len(ref.utils.color_table), "colours,", len(ext), "views")


if __name__ == "__main__":
    main()
