"""MI355X-native ``reconstruct`` package: the DeepSDF shape-prior hot path of DSP-SLAM.

Drop-in for the reference's ``reconstruct.utils`` (get_configs / get_decoder) and
``reconstruct.optimizer`` (Optimizer / MeshExtractor) as called from the C++ side
through pybind11 (src/System.cc:93-99, src/LocalMapping.cc:38-40).

Data ingest (KITTI / Redwood sequences, mmdet detectors — reference
``reconstruct/{kitti,mono}_sequence.py``, ``detector{2,3}d.py``) is out of scope
(SURVEY.md §2 rows 9-12).  When ``DSR_REFERENCE_RECONSTRUCT`` points at the
reference's ``reconstruct/`` directory, ``get_sequence`` / ``get_detectors`` (same
dispatch as the reference's ``reconstruct/__init__.py:1-22``) load exactly those four
named ingest modules from there.  The host helpers they import from this package exist
here (``reconstruct.loss_utils.get_rays / get_time``, ``reconstruct.utils.read_calib_file /
load_velo_scan / ForceKeyErrorDict``).  Nothing else is ever resolved outside this package:
a missing ``reconstruct.<name>`` (e.g. ``loss``) is an ImportError, never the
reference's torch code.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_INGEST = ("kitti_sequence", "mono_sequence", "detector2d", "detector3d")


def _ingest(name):
    """reconstruct.<name> for one of the out-of-scope ingest modules (_INGEST)."""
    if name not in _INGEST:
        raise ImportError(name)
    full = f"{__name__}.{name}"
    if full in _sys.modules:
        return _sys.modules[full]
    ref = _os.environ.get("DSR_REFERENCE_RECONSTRUCT")
    path = _os.path.join(ref, name + ".py") if ref else None
    if not path or not _os.path.isfile(path):
        raise ImportError(f"{full} is data ingest, outside this package (SURVEY.md §2); point "
                          "DSR_REFERENCE_RECONSTRUCT at a directory providing it")
    spec = _ilu.spec_from_file_location(full, path)
    mod = _ilu.module_from_spec(spec)
    _sys.modules[full] = mod
    spec.loader.exec_module(mod)
    return mod


def get_detectors(configs):
    if configs.detect_online:
        get_detector2d = _ingest("detector2d").get_detector2d
        if configs.data_type == "KITTI":
            return get_detector2d(configs), _ingest("detector3d").get_detector3d(configs)
        return get_detector2d(configs)
    if configs.data_type == "KITTI":
        return None, None
    return None


def get_sequence(data_dir, configs):
    if configs.data_type == "KITTI":
        return _ingest("kitti_sequence").KITIISequence(data_dir, configs)
    if configs.data_type in ("Redwood", "Freiburg"):
        return _ingest("mono_sequence").MonoSequence(data_dir, configs)
    return None
