"""Drop-in for models/inverse_warp.py:121-153 (`inverse_warp`) backed by the
HIP warp kernel; PSNet / PANet / REGNet / REG2D call it once per depth plane."""
from sfm_amd.sweep import check_sizes, inverse_warp  # noqa: F401
