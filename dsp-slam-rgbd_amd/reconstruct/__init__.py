"""MI355X-native ``reconstruct`` package: the DeepSDF shape-prior hot path of DSP-SLAM.

Drop-in for the reference's ``reconstruct.utils`` (get_configs / get_decoder) and
``reconstruct.optimizer`` (Optimizer / MeshExtractor) as called from the C++ side
through pybind11 (src/System.cc:93-99, src/LocalMapping.cc:38-40).

Data ingest (KITTI / Redwood sequences, mmdet detectors — reference
``reconstruct/{kitti,mono}_sequence.py``, ``detector{2,3}d.py``) is out of scope
(SURVEY.md §2 rows 9-12).  When ``DSR_REFERENCE_RECONSTRUCT`` points at the
reference's ``reconstruct/`` directory it is appended to this package's search path,
so ``get_sequence`` / ``get_detectors`` (same dispatch as the reference's
``reconstruct/__init__.py:1-22``) load those modules from there while the hot-path
modules (optimizer, utils) keep resolving here first.
"""
import os as _os

_ref = _os.environ.get("DSR_REFERENCE_RECONSTRUCT")
if _ref and _os.path.isdir(_ref) and _ref not in __path__:
    __path__.append(_ref)


def get_detectors(configs):
    if configs.detect_online:
        from .detector2d import get_detector2d
        if configs.data_type == "KITTI":
            from .detector3d import get_detector3d
            return get_detector2d(configs), get_detector3d(configs)
        return get_detector2d(configs)
    if configs.data_type == "KITTI":
        return None, None
    return None


def get_sequence(data_dir, configs):
    if configs.data_type == "KITTI":
        from .kitti_sequence import KITIISequence
        return KITIISequence(data_dir, configs)
    if configs.data_type in ("Redwood", "Freiburg"):
        from .mono_sequence import MonoSequence
        return MonoSequence(data_dir, configs)
    return None
