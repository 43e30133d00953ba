"""Host-side logic of the drop-in package on CPU (no GPU, no compute calls).

* the entry path the C++ side takes first (System.cc:95-98): ``get_configs`` on a
  config JSON with the reference's keys, then ``config_decoder``'s file handling
  (specs.json + ModelParameters/latest.pth, weights_only) — the device upload itself
  is covered by tests/test_gpu_api.py::test_entry_path_as_the_cpp_side_calls_it;
* argument validation before anything reaches C (a short code would be an
  out-of-bounds read there: the ABI copies code_len floats);
* the ingest hook resolves only the four named data-ingest modules;
* golden F9 (tests/golden/make_mesher.py): the reference's voxel grid and its vertex
  transform around marching cubes.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import pytest

import synthetic as S
from conftest import golden


def _reference_style_config(tmp_path, deepsdf_dir, data_type="Redwood"):
    """A config with the keys configs/config_redwood_01053.json carries (written here)."""
    cfg = {"data_type": data_type, "detect_online": False, "DeepSDF_DIR": str(deepsdf_dir),
           "voxels_dim": 32, "min_bb_area": 1600, "min_mask_area": 1000, "downsample_ratio": 4.0,
           "optimizer": S.REDWOOD_OPTIM, "viewer": {"distance": 10, "tilt": 30, "frame_size": 0.5}}
    p = tmp_path / "config.json"
    p.write_text(json.dumps(cfg))
    return str(p)


def test_get_configs_and_checkpoint_files(tmp_path, full_state, full_layers):
    from deep_sdf.workspace import fold_state, load_specs, model_params_subdir
    from reconstruct.utils import get_configs

    exp = S.write_experiment_dir(str(tmp_path / "deepsdf"), full_state)
    cfg = get_configs(_reference_style_config(tmp_path, exp))
    assert cfg.optimizer.code_len == 64 and cfg.voxels_dim == 32
    assert cfg.optimizer.joint_optim.k3 == S.REDWOOD_OPTIM["joint_optim"]["k3"]
    with pytest.raises(KeyError):
        cfg.no_such_key                      # ForceKeyErrorDict (utils.py:82-84)
    specs = load_specs(cfg.DeepSDF_DIR)
    assert specs["CodeLength"] == 64
    import torch

    saved = torch.load(os.path.join(exp, model_params_subdir, "latest.pth"), map_location="cpu",
                       weights_only=True)
    layers = fold_state(saved["model_state_dict"], specs)
    for (W, b), (W0, b0) in zip(layers, full_layers):
        assert np.array_equal(W, W0) and np.array_equal(b, b0)


class _FakeDecoder:
    code_len = 64
    ctx = None
    handle = None


def test_short_code_is_rejected_before_c():
    from reconstruct.optimizer import MeshExtractor, Optimizer, sdf_eval
    from reconstruct.utils import ForceKeyErrorDict

    opt = Optimizer(_FakeDecoder(), ForceKeyErrorDict(data_type="KITTI", optimizer=S.KITTI_OPTIM))
    ob = S.redwood_object(0, n_pts=16)
    short = np.zeros(10, np.float32)
    with pytest.raises(ValueError):
        opt.reconstruct_objects([(ob.t_cam_obj, ob.pts, ob.rays, ob.depth, short)])
    with pytest.raises(ValueError):
        opt.estimate_pose_cam_obj(ob.t_cam_obj, 1.0, ob.pts, short)
    with pytest.raises(ValueError):
        opt.estimate_pose_cam_obj_batch([(ob.t_cam_obj, 1.0, ob.pts, short)])
    with pytest.raises(ValueError):
        opt.compute_sdf_loss_objectpoint_zhjd(ob.pts, short)
    with pytest.raises(ValueError):
        sdf_eval(_FakeDecoder(), short, ob.pts)
    mex = MeshExtractor.__new__(MeshExtractor)          # no device grid upload
    mex.decoder, mex.code_len = _FakeDecoder(), 64
    with pytest.raises(ValueError):
        mex.extract_mesh_from_code(short)


def test_ingest_hook_resolves_only_named_modules(tmp_path, monkeypatch):
    import reconstruct
    from reconstruct.utils import ForceKeyErrorDict

    (tmp_path / "mono_sequence.py").write_text(
        "class MonoSequence:\n    def __init__(self, d, c):\n        self.d = d\n")
    (tmp_path / "loss.py").write_text("raise RuntimeError('must never be imported')\n")
    monkeypatch.setenv("DSR_REFERENCE_RECONSTRUCT", str(tmp_path))
    monkeypatch.delitem(sys.modules, "reconstruct.mono_sequence", raising=False)
    seq = reconstruct.get_sequence("/data", ForceKeyErrorDict(data_type="Redwood"))
    assert seq.d == "/data"
    with pytest.raises(ImportError):
        import reconstruct.loss  # noqa: F401
    assert reconstruct.get_detectors(ForceKeyErrorDict(detect_online=False, data_type="KITTI")) == (None, None)
    monkeypatch.delitem(sys.modules, "reconstruct.mono_sequence", raising=False)


def test_voxel_grid_matches_reference_f9():
    from reconstruct.utils import create_voxel_grid

    f = golden("f9_mesher.npz")
    g = create_voxel_grid(vol_dim=int(f["dim"]))
    assert g.dtype == np.float32 and np.array_equal(g, f["grid"])


def test_vertex_transform_matches_reference_f9():
    from oracle.dsr_mc import vertex_transform

    f = golden("f9_mesher.npz")
    assert str(f["verts_dtype"]) == "float32"
    assert np.array_equal(vertex_transform(f["verts_index"], int(f["dim"])), f["verts_out"])
    assert np.allclose(f["spacing"], 2.0 / (int(f["dim"]) - 1)) and float(f["level"]) == 0.0


def test_grid_decode_order_matches_reference_f9(oracle_dec):
    """The reference decodes create_voxel_grid's points and views them as (d, d, d)
    (optimizer.py:225-227): the oracle's decode in the same order reproduces the volume."""
    from oracle import dsr_oracle as O
    from reconstruct.utils import create_voxel_grid

    f = golden("f9_mesher.npz")
    d = int(f["dim"])
    vol = O.decode_sdf(oracle_dec, f["code"], create_voxel_grid(vol_dim=d)).reshape(d, d, d)
    assert np.abs(vol - f["volume"]).max() <= 2e-5


@pytest.mark.parametrize("change,what", [
    ({"weight_norm": False}, "LayerNorm"),
    ({"xyz_in_all": True}, "xyz_in_all"),
    ({"use_tanh": True}, "use_tanh"),
    ({"latent_in": [3]}, "latent_in"),
])
def test_unsupported_decoder_variants_rejected_loudly(change, what):
    """decoder variants libdsr does not implement (deep_sdf_decoder.py:46-47,
    58-67, 89-102) are refused before anything reaches the device, never approximated."""
    import copy

    import synthetic as S
    from deep_sdf.workspace import check_topology, fold_state

    layers = fold_state(S.make_decoder(1234), S.DEFAULT_SPECS)
    check_topology(S.DEFAULT_SPECS, layers)                  # the supported topology passes
    specs = copy.deepcopy(S.DEFAULT_SPECS)
    specs["NetworkSpecs"].update(change)
    with pytest.raises(NotImplementedError, match=what):
        check_topology(specs, layers)
    specs = copy.deepcopy(S.DEFAULT_SPECS)
    specs["CodeLength"] = 32
    with pytest.raises(NotImplementedError, match="CodeLength"):
        check_topology(specs, layers)
