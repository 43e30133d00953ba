"""Config / decoder factory half of ``reconstruct/utils.py`` (utils.py:82-116).

Same names and behaviour the C++ side relies on (src/System.cc:95-98):
``get_configs(path)`` returns an attribute dict that raises ``KeyError`` on a
missing key (``ForceKeyErrorDict``, utils.py:82-90), ``get_decoder(cfg)`` returns
the decoder handle built from ``cfg.DeepSDF_DIR`` (utils.py:93-94).
"""
from __future__ import annotations

import json

import numpy as np


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
