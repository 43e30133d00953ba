"""Shared test fixtures.

``-m "not gpu"``: oracle vs golden vectors, host logic, C-ABI load/exports (CPU).
``-m gpu``: HIP path (libdsr.so through ctypes) vs the oracle / golden vectors on a
real MI355X.  GPU tests never fall back: a missing library or device fails them.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "dsp-slam-rgbd_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import synthetic as S  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built libdsr.so")
    config.addinivalue_line("markers", "slow: longer CPU test")


def golden(name):
    path = os.path.join(GOLDEN, name)
    return np.load(path, allow_pickle=False)


@pytest.fixture(scope="session")
def full_state():
    return S.make_decoder(1234)


@pytest.fixture(scope="session")
def full_layers(full_state):
    from deep_sdf.workspace import fold_state

    return fold_state(full_state, S.DEFAULT_SPECS)


@pytest.fixture(scope="session")
def oracle_dec(full_layers):
    from oracle.dsr_oracle import Decoder

    return Decoder(full_layers, 64, (4,))


@pytest.fixture(scope="session")
def gpu_decoder(full_state):
    from deep_sdf.workspace import decoder_from_state

    return decoder_from_state(full_state, S.DEFAULT_SPECS)


def make_cfg(optim, data_type="KITTI"):
    from reconstruct.utils import ForceKeyErrorDict

    return ForceKeyErrorDict(data_type=data_type, optimizer=optim)


def assert_jac_close(j, jref, tol=2e-5, loose=5e-2, frac=0.01):
    """Jacobian rows agree to ``tol`` (x max|jref|) except for at most max(2, frac*n)
    points — those with a hidden pre-activation within rounding of 0, where fp32 vs
    the reference decides the ReLU mask by the last bit — which stay within ``loose``."""
    j = np.asarray(j, np.float64)
    jref = np.asarray(jref, np.float64)
    scale = max(1.0, float(np.abs(jref).max()))
    per_pt = np.abs(j - jref).max(axis=1) / scale
    n_bad = int((per_pt > tol).sum())
    assert n_bad <= max(2, int(frac * per_pt.shape[0])), (per_pt.max(), n_bad)
    assert per_pt.max() <= loose, per_pt.max()
