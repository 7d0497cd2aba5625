"""orb_slam_cuda_amd — MI355X-native ORB front-end for ORB-SLAM2.

The hot path of falfab/orb_slam_cuda (ORBextractor::operator() and the
ORBmatcher searches SearchForInitialization / SearchByBoW) as hand-written
HIP kernels for gfx950 behind a C ABI (include/orbx_c.h, liborbx.so), with a
host-side mirror of the reference classes in Python.
"""
from ._lib import KP_DTYPE, OrbxError, device_count, header_functions, lib  # noqa: F401
from .extractor import ORBextractor  # noqa: F401
from .matcher import ComputeStereoMatches, ComputeStereoMatchesLast, ExtractStereo, Frame, KeyFrame, MapPoints, ORBmatcher  # noqa: F401
from .vocabulary import ComputeBoW, ORBVocabulary  # noqa: F401

__all__ = ["ORBextractor", "ORBmatcher", "ORBVocabulary", "Frame", "KeyFrame", "ComputeBoW",
           "ComputeStereoMatches", "ComputeStereoMatchesLast", "ExtractStereo", "MapPoints", "KP_DTYPE", "OrbxError",
           "device_count", "header_functions", "lib"]
