"""Loader for the HIP product library liborbx.so (built in-tree by build()).

There is no CPU fallback: if the library or a gfx950 device is missing,
every entry point raises. The ctypes signatures mirror include/orbx_c.h.
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORBX_LIB_VARIANT=<name> loads variants/liborbx_<name>.so (tools/variant.sh
# builds them: a kernel compiled with other tuning constants, for A/B timing)
LIB_PATH = os.path.join(HERE, "liborbx.so")
if os.environ.get("ORBX_LIB_VARIANT"):
    LIB_PATH = os.path.join(HERE, "variants", "liborbx_%s.so" % os.environ["ORBX_LIB_VARIANT"])
HEADER = os.path.join(os.path.dirname(HERE), "include", "orbx_c.h")

ORBX_OK, ORBX_EINVAL, ORBX_EDEVICE, ORBX_ECAPACITY, ORBX_ENOMEM = 0, -1, -2, -3, -4

# cv::KeyPoint layout (include/orbx_c.h orbx_kp)
KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KP_DTYPE.itemsize == 28


class OrbxConfig(C.Structure):
    _fields_ = [("nfeatures", C.c_int), ("scale_factor", C.c_float), ("nlevels", C.c_int),
                ("ini_th_fast", C.c_int), ("min_th_fast", C.c_int), ("width", C.c_int),
                ("height", C.c_int), ("device", C.c_int), ("max_batch", C.c_int),
                ("scale_mode", C.c_int), ("pattern_mode", C.c_int), ("reserved", C.c_int * 5)]


class GridBounds(C.Structure):
    _fields_ = [("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float), ("max_y", C.c_float)]


class OrbmCamera(C.Structure):
    """orbm_camera: fx, fy, cx, cy, mb, mbf and mTcw rows 0..2 (row-major)."""
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("mb", C.c_float), ("mbf", C.c_float), ("Tcw", C.c_float * 12)]


class OrbmPose(C.Structure):
    """orbm_pose (orbm_prepare_pose / orbm_prepare_sim3_match), 132 bytes."""
    _fields_ = [("Rt", C.c_float * 12), ("Ow", C.c_float * 3), ("fx", C.c_float), ("fy", C.c_float),
                ("cx", C.c_float), ("cy", C.c_float), ("mbf", C.c_float), ("level_mode", C.c_int32),
                ("Rt2", C.c_float * 12)]


assert C.sizeof(OrbmPose) == 132


class OrbmTriPair(C.Structure):
    """orbm_tri_pair (orbm_prepare_triangulation), 44 bytes."""
    _fields_ = [("F12", C.c_float * 9), ("ex", C.c_float), ("ey", C.c_float)]


def camera(fx, fy, cx, cy, mb, mbf, Tcw) -> OrbmCamera:
    T = np.asarray(Tcw, np.float32).reshape(-1)[:12]
    return OrbmCamera(fx, fy, cx, cy, mb, mbf, (C.c_float * 12)(*T.tolist()))


class FeatureVectorC(C.Structure):
    _fields_ = [("nodes", C.c_void_p), ("off", C.c_void_p), ("idx", C.c_void_p), ("n_nodes", C.c_int)]


class OrbxError(RuntimeError):
    """Raised for any non-zero status (the reference throws std::runtime_error)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"orbx error {code}: {msg}")
        self.code = code


_lib = None


class _Tolerant:
    """A loaded library whose missing symbols read as throwaway objects, so the
    signature table below can be applied to an older variant build."""

    def __init__(self, L):
        self.__dict__["_L"] = L

    def __getattr__(self, name):
        try:
            return getattr(self._L, name)
        except AttributeError:
            return type("Missing", (), {})()


def stage_order(handle=None) -> list:
    """The extraction stages in launch order of an extractor handle (None: the
    default), as bench.py's stage names (orbx_get_stage_order): stage event
    i + 1 closes entry i."""
    buf = C.create_string_buffer(6)
    check(lib().orbx_get_stage_order(handle, buf))
    names = {"p": "pyramid", "b": "blur", "f": "fast_grid", "q": "quadtree", "o": "orient_brief"}
    return [names[c] for c in buf.value.decode()]


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OrbxError(ORBX_EDEVICE, f"{LIB_PATH} not built; run __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        if os.environ.get("ORBX_LIB_VARIANT"):
            # A/B builds of other revisions may lack newer entry points: their
            # signatures are skipped here (a call to one fails when made)
            L = _Tolerant(L)
        L.orbx_last_error.restype = C.c_char_p
        L.orbm_last_error.restype = C.c_char_p
        L.orbx_version.restype = C.c_char_p
        L.orbx_create.argtypes = [C.POINTER(OrbxConfig), C.POINTER(C.c_void_p)]
        for name in ("orbx_destroy", "orbx_frame_capacity"):
            getattr(L, name).argtypes = [C.c_void_p]
        L.orbx_extract.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_size_t, C.c_void_p,
                                   C.c_int, C.c_void_p, C.POINTER(C.c_int)]
        L.orbx_extract_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_size_t, C.c_size_t,
                                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orbx_get_scales.argtypes = [C.c_void_p] + [C.c_void_p] * 4
        L.orbx_get_levels_info.argtypes = [C.c_void_p] + [C.c_void_p] * 4
        L.orbx_get_stage_order.argtypes = [C.c_void_p, C.c_char_p]
        L.orbx_set_stage_order.argtypes = [C.c_void_p, C.c_char_p]
        L.orbx_get_level.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_size_t]
        L.orbx_set_host_pyramid.argtypes = [C.c_void_p, C.c_int]
        L.orbx_get_host_pyramid.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.orbx_get_fast_candidates.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                               C.POINTER(C.c_int)]
        L.orbx_get_stage_times.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_int)]
        L.orbx_set_stage_events.argtypes = [C.c_void_p, C.c_void_p]
        L.orbx_get_tie_stats.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        L.orbx_get_quadtree_paths.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        L.orbx_get_status.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int)]
        L.orbx_get_pattern.argtypes = [C.c_int, C.c_void_p]
        L.orbm_get_status.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int)]
        L.orbm_create.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
        L.orbm_destroy.argtypes = [C.c_void_p]
        L.orbm_descriptor_distance.argtypes = [C.c_void_p, C.c_void_p]
        L.orbm_hamming_top2.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_int,
                                        C.c_void_p, C.c_size_t, C.c_void_p, C.c_int, C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_void_p]
        L.orbm_search_for_initialization.argtypes = [
            C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int, GridBounds,
            C.c_void_p, C.c_int, C.c_float, C.c_int, C.c_void_p, C.POINTER(C.c_int)]
        L.orbm_search_for_initialization_batch.argtypes = [
            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
            C.c_int, GridBounds, C.c_void_p, C.c_int, C.c_float, C.c_int, C.c_void_p, C.c_void_p,
            C.c_void_p]
        L.orbm_search_by_bow.argtypes = [
            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, FeatureVectorC, C.c_void_p,
            C.c_void_p, C.c_void_p, C.c_int, FeatureVectorC, C.c_float, C.c_int, C.c_int, C.c_void_p,
            C.POINTER(C.c_int)]
        L.orbm_search_by_bow_batch.argtypes = ([C.c_void_p, C.c_int, C.c_int, C.c_int] + [C.c_void_p] * 16
                                               + [C.c_float, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p])
        L.orbm_compute_stereo_matches.argtypes = [
            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
            C.c_int, C.c_float, C.c_float, C.c_void_p, C.c_void_p, C.POINTER(C.c_int)]
        L.orbm_compute_stereo_matches_last.argtypes = [
            C.c_void_p, C.c_void_p, C.c_void_p, C.c_float, C.c_float, C.c_void_p, C.c_void_p, C.c_int,
            C.POINTER(C.c_int)]
        L.orbm_stereo_frame.argtypes = [
            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int, C.c_int,
            C.c_float, C.c_float, C.c_void_p, C.c_int, C.c_void_p, C.POINTER(C.c_int), C.c_void_p, C.c_int,
            C.c_void_p, C.POINTER(C.c_int), C.c_void_p, C.c_void_p, C.POINTER(C.c_int)]
        L.orbm_compute_stereo_matches_batch.argtypes = [
            C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
            C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_float, C.c_float, C.c_void_p,
            C.c_void_p, C.c_void_p, C.c_void_p]
        L.orbm_search_by_projection.argtypes = ([C.c_void_p] * 3 + [C.c_int, C.c_void_p, GridBounds, C.c_void_p,
                                                 C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_float,
                                                 C.c_float, C.c_void_p, C.POINTER(C.c_int)])
        L.orbm_search_by_projection_batch.argtypes = ([C.c_void_p] * 4 + [C.c_int, C.c_void_p, GridBounds,
                                                       C.c_void_p, C.c_int] + [C.c_void_p] * 4
                                                      + [C.c_int, C.c_int, C.c_float, C.c_float] + [C.c_void_p] * 3)
        PS = [C.c_void_p] * 3 + [C.c_int]  # handle, kps, desc, n
        L.orbm_prepare_pose.argtypes = [C.c_int, C.POINTER(OrbmCamera), C.c_void_p, C.c_int, C.POINTER(OrbmPose)]
        L.orbm_predict_scale_thresholds.argtypes = [C.c_float, C.c_int, C.c_void_p]
        L.orbm_predict_scale.argtypes = [C.c_float, C.c_float, C.c_float, C.c_int]
        L.orbm_search_by_projection_last_frame.argtypes = (
            PS + [C.c_void_p, GridBounds, C.c_void_p, C.c_int, C.c_void_p, C.POINTER(OrbmCamera), C.c_void_p,
                  C.c_void_p, C.c_void_p, C.c_int, C.c_float, C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_int)])
        L.orbm_search_by_projection_keyframe.argtypes = (
            PS + [GridBounds, C.c_void_p, C.c_int, C.c_float, C.c_void_p, C.POINTER(OrbmCamera), C.c_void_p,
                  C.c_void_p, C.c_int, C.c_float, C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_int)])
        L.orbm_search_by_projection_sim3.argtypes = (
            PS + [GridBounds, C.c_void_p, C.c_int, C.c_float, C.POINTER(OrbmCamera), C.c_void_p, C.c_void_p,
                  C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_int)])
        L.orbm_search_by_projection_pose_batch.argtypes = (
            [C.c_void_p, C.c_int] + [C.c_void_p] * 3 + [C.c_int, C.c_void_p, GridBounds, C.c_void_p, C.c_int,
                                                         C.c_float] + [C.c_void_p] * 5
            + [C.c_int, C.c_int, C.c_float, C.c_int, C.c_int] + [C.c_void_p] * 4)
        L.orbm_prepare_sim3_match.argtypes = [C.POINTER(OrbmCamera), C.c_void_p, C.c_void_p, C.c_float, C.c_void_p,
                                              C.c_void_p, C.POINTER(OrbmPose)]
        L.orbm_fuse.argtypes = (PS + [C.c_void_p, GridBounds, C.c_void_p, C.c_void_p, C.c_int, C.c_float,
                                      C.POINTER(OrbmCamera), C.c_void_p, C.c_void_p, C.c_int, C.c_float, C.c_void_p,
                                      C.POINTER(C.c_int)])
        L.orbm_fuse_sim3.argtypes = (PS + [GridBounds, C.c_void_p, C.c_int, C.c_float, C.POINTER(OrbmCamera),
                                           C.c_void_p, C.c_void_p, C.c_int, C.c_float, C.c_void_p,
                                           C.POINTER(C.c_int)])
        L.orbm_search_by_sim3.argtypes = (PS + [GridBounds, C.c_void_p, C.c_void_p, C.c_void_p]
                                          + [C.c_void_p] * 2 + [C.c_int, GridBounds] + [C.c_void_p] * 4
                                          + [C.c_int, C.c_float, C.POINTER(OrbmCamera), C.c_float, C.c_void_p,
                                             C.c_void_p, C.c_float, C.c_void_p, C.POINTER(C.c_int)])
        L.orbm_prepare_triangulation.argtypes = [C.c_void_p] * 4 + [C.POINTER(OrbmTriPair)]
        L.orbm_search_for_triangulation.argtypes = (
            [C.c_void_p] * 5 + [C.c_int, FeatureVectorC] + [C.c_void_p] * 4 + [C.c_int, FeatureVectorC]
            + [C.c_void_p] * 5 + [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_int)])
        L.orbm_search_for_triangulation_batch.argtypes = (
            [C.c_void_p] + ([C.c_void_p] * 9 + [C.c_int, C.c_int]) * 2 + [C.c_void_p] * 3
            + [C.c_int] * 4 + [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p])
        L.orbv_last_error.restype = C.c_char_p
        L.orbv_load_text.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_void_p)]
        L.orbv_create.argtypes = [C.c_int] * 5 + [C.c_void_p] * 4 + [C.c_int, C.POINTER(C.c_void_p)]
        L.orbv_destroy.argtypes = [C.c_void_p]
        L.orbv_info.argtypes = [C.c_void_p] + [C.POINTER(C.c_int)] * 6
        L.orbv_transform.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int] + [C.c_void_p] * 10
        L.orbv_transform_batch.argtypes = ([C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_int, C.c_int,
                                            C.c_int] + [C.c_void_p] * 11)
        L.orbx_device_count.argtypes = [C.POINTER(C.c_int)]
        L.orbx_set_device.argtypes = [C.c_int]
        L.orbx_malloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        L.orbx_free.argtypes = [C.c_void_p]
        L.orbx_memcpy_htod.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.orbx_memcpy_dtoh.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.orbx_memset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
        L.orbx_memcpy_dtod_async.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.orbx_memcpy_htod_async.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.orbx_memcpy_dtoh_async.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.orbx_memcpy2d_htod_async.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t,
                                               C.c_size_t, C.c_void_p]
        L.orbx_copy2d_kernel_async.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t,
                                               C.c_size_t, C.c_int, C.c_void_p]
        L.orbx_host_alloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        L.orbx_host_free.argtypes = [C.c_void_p]
        L.orbx_stream_create.argtypes = [C.POINTER(C.c_void_p)]
        L.orbx_stream_create_priority.argtypes = [C.POINTER(C.c_void_p), C.c_int]
        L.orbx_stream_destroy.argtypes = [C.c_void_p]
        L.orbx_stream_synchronize.argtypes = [C.c_void_p]
        L.orbx_event_create.argtypes = [C.POINTER(C.c_void_p)]
        L.orbx_event_destroy.argtypes = [C.c_void_p]
        L.orbx_event_record.argtypes = [C.c_void_p, C.c_void_p]
        L.orbx_event_elapsed_ms.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_float)]
        L.orbx_stream_wait_event.argtypes = [C.c_void_p, C.c_void_p]
        L.orbx_sincosf_glibc.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


# orbm_map_point_world (include/orbx_c.h), 48 bytes
MAP_POINT_WORLD_DTYPE = np.dtype([("pos", "<f4", (3,)), ("normal", "<f4", (3,)), ("min_distance", "<f4"),
                                  ("max_distance", "<f4"), ("angle", "<f4"), ("octave", "<i4"), ("valid", "u1"),
                                  ("obs_positive", "u1"), ("pad", "u1", (6,))])
assert MAP_POINT_WORLD_DTYPE.itemsize == 48
ORBM_PROJ_LAST_FRAME, ORBM_PROJ_KEYFRAME, ORBM_PROJ_SIM3 = 1, 2, 3
ORBM_PROJ_FUSE, ORBM_PROJ_FUSE_SIM3, ORBM_PROJ_SIM3_MATCH = 4, 5, 6

# orbm_map_point_proj (include/orbx_c.h), 24 bytes
MAP_POINT_PROJ_DTYPE = np.dtype([("proj_x", "<f4"), ("proj_y", "<f4"), ("proj_xr", "<f4"), ("view_cos", "<f4"),
                                 ("predicted_level", "<i4"), ("track_in_view", "u1"), ("obs_positive", "u1"),
                                 ("pad", "u1", (2,))])


def check(rc: int, matcher: bool = False, vocabulary: bool = False) -> None:
    if rc != ORBX_OK:
        L = lib()
        msg = (L.orbv_last_error() if vocabulary else
               L.orbm_last_error() if matcher else L.orbx_last_error()) or b""
        raise OrbxError(rc, msg.decode(errors="replace"))


def header_functions(path: str = HEADER) -> list[str]:
    """Names of every function declared in include/orbx_c.h."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b((?:orbx|orbm|orbv)_[a-z0-9_]+)\s*\(", src)))


def ptr(a) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data) if a is not None else C.c_void_p(0)


def device_count() -> int:
    n = C.c_int(0)
    check(lib().orbx_device_count(C.byref(n)))
    return n.value


class DeviceArray:
    """Owning device allocation (hipMalloc through the C ABI)."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        self.p = C.c_void_p(0)
        check(lib().orbx_malloc(C.byref(self.p), max(self.nbytes, 1)))

    @property
    def ptr(self) -> int:
        return self.p.value

    def upload(self, a: np.ndarray, offset: int = 0) -> None:
        a = np.ascontiguousarray(a)
        assert offset + a.nbytes <= self.nbytes
        check(lib().orbx_memcpy_htod(C.c_void_p(self.ptr + offset), ptr(a), a.nbytes))

    def download(self, shape, dtype, offset: int = 0) -> np.ndarray:
        out = np.empty(shape, dtype)
        assert offset + out.nbytes <= self.nbytes
        check(lib().orbx_memcpy_dtoh(ptr(out), C.c_void_p(self.ptr + offset), out.nbytes))
        return out

    def zero(self) -> None:
        check(lib().orbx_memset(self.p, 0, self.nbytes))

    def __del__(self):
        if getattr(self, "p", None) and self.p.value and _lib is not None:
            _lib.orbx_free(self.p)
            self.p = C.c_void_p(0)


class HostArray:
    """Owning pinned host allocation (hipHostMalloc) viewed as a numpy array."""

    def __init__(self, shape, dtype):
        self.dtype = np.dtype(dtype)
        self.shape = tuple(shape) if isinstance(shape, (tuple, list)) else (int(shape),)
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        self.p = C.c_void_p(0)
        check(lib().orbx_host_alloc(C.byref(self.p), max(self.nbytes, 1)))
        buf = (C.c_uint8 * max(self.nbytes, 1)).from_address(self.p.value)
        self.a = np.frombuffer(buf, np.uint8, self.nbytes).view(self.dtype).reshape(self.shape)

    @property
    def ptr(self) -> int:
        return self.p.value

    def __del__(self):
        if getattr(self, "p", None) and self.p.value and _lib is not None:
            self.a = None
            _lib.orbx_host_free(self.p)
            self.p = C.c_void_p(0)


class Stream:
    def __init__(self, priority: int | None = None, cu_mask: list | None = None):
        """priority None: default; 1: preferred by the dispatcher; 0: deferred.
        cu_mask: list of u32 words, the compute units the stream may use."""
        self.s = C.c_void_p(0)
        if cu_mask is not None:
            m = (C.c_uint32 * len(cu_mask))(*cu_mask)
            check(lib().orbx_stream_create_cumask(C.byref(self.s), m, len(cu_mask)))
        elif priority is None:
            check(lib().orbx_stream_create(C.byref(self.s)))
        else:
            check(lib().orbx_stream_create_priority(C.byref(self.s), int(priority)))

    def synchronize(self) -> None:
        check(lib().orbx_stream_synchronize(self.s))

    def wait(self, event: "Event") -> None:
        check(lib().orbx_stream_wait_event(self.s, event.e))

    def __del__(self):
        if getattr(self, "s", None) and self.s.value and _lib is not None:
            _lib.orbx_stream_destroy(self.s)


class Event:
    def __init__(self):
        self.e = C.c_void_p(0)
        check(lib().orbx_event_create(C.byref(self.e)))

    def record(self, stream: Stream) -> None:
        check(lib().orbx_event_record(self.e, stream.s))

    def elapsed_ms(self, end: "Event") -> float:
        ms = C.c_float(0)
        check(lib().orbx_event_elapsed_ms(self.e, end.e, C.byref(ms)))
        return ms.value

    def __del__(self):
        if getattr(self, "e", None) and self.e.value and _lib is not None:
            _lib.orbx_event_destroy(self.e)
