"""stereo_matchin_amd — MI355X-native adaptive-support-weight stereo matcher.

A drop-in for the OpenCL ``kernels/`` ASW path of manixq/stereo_matchin
(stereo_matching/main.cpp:413-537): hand-written gfx950 HIP kernels behind the
C-ABI in ``include/asw.h`` (``libasw_hip.so``), a Python mirror of the
reference's kernel interface (:mod:`.kernels`), the one-GPU pipeline
(:mod:`.pipeline`) and disparity-axis sharding over RCCL (:mod:`.distributed`).
"""
from ._lib import (ASW_OK, COLOR_LAB, COLOR_RGB, DIR_H, DIR_V, LR_NATIVE, LR_U8, AswError,  # noqa: F401
                   AswLibraryError, AswParams, default_params)
from .pipeline import (FrameContext, MatchResult, StereoMatcher, comm_unique_id, make_params,  # noqa: F401
                       match_frame, to_rgba)

__all__ = [
    "AswParams", "AswError", "AswLibraryError", "StereoMatcher", "MatchResult", "make_params", "match_frame",
    "FrameContext", "comm_unique_id",
    "to_rgba", "default_params",
]
