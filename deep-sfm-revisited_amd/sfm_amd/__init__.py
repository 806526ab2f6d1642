"""sfm_amd — MI355X-native hot path of two-view deep SfM (jytime/Deep-SfM-Revisited).

Host-side mirror of the reference's operator interfaces over the C ABI of
libsfm_hip.so (include/sfm_hip.h):
  ransac   batched RANSAC five-point (essential_matrix extension), flow -> points
  sweep    plane-sweep cost volume, inverse_warp, PSNet sweep section
  regularize  PSNet 3-D cost regularisation (dres0..classify) on the matrix cores
  synth    seeded synthetic KITTI-shaped inputs
  dist     one-process-per-GPU pair sharding and RCCL metric gather
"""
from . import _lib  # noqa: F401

__all__ = ["ransac", "sweep", "regularize", "synth", "dist", "config"]
