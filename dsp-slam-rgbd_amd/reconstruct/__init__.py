"""MI355X-native ``reconstruct`` package: the DeepSDF shape-prior hot path of DSP-SLAM.

Drop-in for the reference's ``reconstruct.utils`` (get_configs / get_decoder) and
``reconstruct.optimizer`` (Optimizer / MeshExtractor) as called from the C++ side
through pybind11.  Data ingest (KITTI / Redwood sequences, mmdet detectors:
reference ``reconstruct/__init__.py:1-22``) is out of scope.
"""
