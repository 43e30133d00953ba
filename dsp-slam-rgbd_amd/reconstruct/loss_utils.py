"""The two HOST helpers of the reference's ``reconstruct/loss_utils.py`` that its data-ingest
modules import (``kitti_sequence.py:22`` / ``mono_sequence.py:22``: ``from
reconstruct.loss_utils import get_rays, get_time``), so that ``reconstruct.get_sequence``
(called at every start-up, src/System.cc:99) works with the reference's own ingest modules.

The rest of that file — decode_sdf, the batched Jacobian, the Sim(3) algebra, Huber — is the
hot path and lives in libdsr's kernels (include/dsr.h); it is deliberately not here.
"""
from __future__ import annotations

import time

import numpy as np


def get_rays(sampled_pixels, invK):
    """loss_utils.py:23-37: ray directions ``[u, v, 1] . invK^T`` (N, 3) float32 in the camera
    frame for (N, 2) pixels ``[u, v]``, with the reference's broadcast-and-sum arithmetic."""
    n = sampled_pixels.shape[0]
    u_hom = np.concatenate([sampled_pixels, np.ones((n, 1))], axis=-1)
    return (u_hom[:, None, :] * invK).sum(-1).astype(np.float32)


def get_time():
    """loss_utils.py:278-283: wall time after the device has drained (the reference calls
    torch.cuda.synchronize(); libdsr's calls are synchronous unless async handles are used)."""
    try:
        import torch

        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except ImportError:
        pass
    return time.time()
