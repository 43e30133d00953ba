"""Mesh extraction from a decoded SDF grid (utils.py:119-140) — SURVEY.md §8f rank 1.

The reference calls ``skimage.measure.marching_cubes_lewiner`` (removed after
scikit-image 0.18; skimage is not installed in this image).  A device marching
cubes is the planned follow-on; until it lands this raises loudly instead of
silently producing a different mesh.
"""


def marching_cubes_lewiner_like(sdf):
    raise NotImplementedError("marching cubes (MeshExtractor.extract_mesh_from_code) is a "
                              "§8f follow-on; MeshExtractor.decode_grid() gives the SDF grid")
