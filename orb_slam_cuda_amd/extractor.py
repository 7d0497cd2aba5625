"""ORBextractor — host-side mirror of ORB_SLAM2::ORBextractor over liborbx.

Same constructor arguments, call signature, getters and error behaviour as
the reference (include/ORBextractor.h:75-197, src/ORBextractor.cc:496-1815):

    ext = ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST,
                       width, height)
    keypoints, descriptors = ext(image)          # operator()(image, mask, kps, desc)
    ext.GetScaleFactors(); ext.mvImagePyramid    # getters / public pyramid

Keypoints come back as a numpy structured array with the cv::KeyPoint field
layout (KP_DTYPE), descriptors as an (N, 32) uint8 array, in the reference
order (level-major, quadtree order inside a level). All computation runs in
the HIP kernels of liborbx.so; nothing here computes features.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import KP_DTYPE, OrbxConfig, check, lib, ptr

SCALE_MODES = {"U": 0, "F": 1}
PATTERNS = {"fork": 0, "upstream": 1}


class ORBextractor:
    HARRIS_SCORE, FAST_SCORE = 0, 1  # include/ORBextractor.h:80 (unused by the reference)

    def __init__(self, nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int,
                 minThFAST: int, width: int, height: int, *, device: int = 0, max_batch: int = 1,
                 scale_mode: str = "U", pattern: str = "fork"):
        cfg = OrbxConfig()
        cfg.nfeatures, cfg.scale_factor, cfg.nlevels = int(nfeatures), float(scaleFactor), int(nlevels)
        cfg.ini_th_fast, cfg.min_th_fast = int(iniThFAST), int(minThFAST)
        cfg.width, cfg.height = int(width), int(height)
        cfg.device, cfg.max_batch = int(device), int(max_batch)
        cfg.scale_mode, cfg.pattern_mode = SCALE_MODES[scale_mode], PATTERNS[pattern]
        self.cfg = cfg
        self._h = C.c_void_p(0)
        check(lib().orbx_create(C.byref(cfg), C.byref(self._h)))
        self.nfeatures, self.scaleFactor, self.nlevels = cfg.nfeatures, cfg.scale_factor, cfg.nlevels
        self.iniThFAST, self.minThFAST = cfg.ini_th_fast, cfg.min_th_fast

    # ------------------------------------------------------------- lifetime
    def close(self) -> None:
        if self._h and self._h.value:
            lib().orbx_destroy(self._h)
            self._h = C.c_void_p(0)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    @property
    def frame_capacity(self) -> int:
        return lib().orbx_frame_capacity(self._h)

    # ------------------------------------------------------------- operator()
    def __call__(self, image: np.ndarray, mask=None):
        """ORBextractor::operator()(image, mask, keypoints, descriptors); mask is ignored
        like the reference (include/ORBextractor.h:89)."""
        img = np.asarray(image)
        if img.size == 0:
            # no outputs (src/ORBextractor.cc:1542-1543); the handle's last
            # extraction becomes an empty one (what the stereo matcher then reads)
            check(lib().orbx_extract(self._h, None, 0, 0, 0, None, 0, None, C.byref(C.c_int(0))))
            return np.zeros(0, KP_DTYPE), np.zeros((0, 32), np.uint8)
        if img.dtype != np.uint8 or img.ndim != 2:
            raise _lib.OrbxError(_lib.ORBX_EINVAL, "image must be CV_8UC1 (2-D uint8)")  # :1546 assert
        if img.strides[1] != 1:
            img = np.ascontiguousarray(img)
        cap = self._begin(img)
        n = C.c_int(0)
        kps = np.empty(cap, KP_DTYPE)
        desc = np.empty((cap, 32), np.uint8)
        check(lib().orbx_extract(self._h, ptr(img), img.shape[1], img.shape[0], img.strides[0],
                                 ptr(kps), cap, ptr(desc), C.byref(n)))
        return kps[:n.value].copy(), desc[:n.value].copy()

    def _begin(self, img: np.ndarray) -> int:
        """Plan the handle for the image's size (created with width/height 0, as mono
        yamls without Camera.width/height leave it, src/Tracking.cc:124-133, or a new
        size: the reference accepts any size per call) with one call that has no
        outputs; returns the frame capacity the outputs are sized to."""
        lw = (C.c_int * self.nlevels)()
        lh = (C.c_int * self.nlevels)()
        nl = C.c_int(0)
        check(lib().orbx_get_levels_info(self._h, C.byref(nl), lw, lh, None))
        if (lw[0], lh[0]) != (img.shape[1], img.shape[0]):
            n = C.c_int(0)
            check(lib().orbx_extract(self._h, ptr(img), img.shape[1], img.shape[0], img.strides[0],
                                     None, 2**31 - 1, None, C.byref(n)))
        return self.frame_capacity

    def set_stage_order(self, order: str) -> None:
        """The stages' launch order for later extractions (orbx_set_stage_order)."""
        check(lib().orbx_set_stage_order(self._h, order.encode()))

    def stage_order(self) -> list:
        return _lib.stage_order(self._h)

    def extract_batch_device(self, d_frames: int, batch: int, frame_pitch: int, row_stride: int,
                             d_kps: int, d_desc: int, d_counts: int, stream=None) -> None:
        """Asynchronous batched extraction on device pointers (orbx_extract_batch)."""
        s = stream.s if stream is not None else C.c_void_p(0)
        check(lib().orbx_extract_batch(self._h, C.c_void_p(d_frames), batch, frame_pitch, row_stride,
                                       C.c_void_p(d_kps), C.c_void_p(d_desc), C.c_void_p(d_counts), s))

    # ------------------------------------------------------------- getters
    def GetLevels(self) -> int:
        return self.nlevels

    def GetScaleFactor(self) -> float:
        return self.scaleFactor

    def _scales(self):
        L = self.nlevels
        a = [np.zeros(L, np.float32) for _ in range(4)]
        check(lib().orbx_get_scales(self._h, *(ptr(x) for x in a)))
        return a

    def GetScaleFactors(self) -> list[float]:
        return self._scales()[0].tolist()

    def GetInverseScaleFactors(self) -> list[float]:
        return self._scales()[1].tolist()

    def GetScaleSigmaSquares(self) -> list[float]:
        return self._scales()[2].tolist()

    def GetInverseScaleSigmaSquares(self) -> list[float]:
        return self._scales()[3].tolist()

    def levels_info(self) -> dict:
        L = self.nlevels
        n = C.c_int(0)
        w, h, nf = (np.zeros(L, np.int32) for _ in range(3))
        check(lib().orbx_get_levels_info(self._h, C.byref(n), ptr(w), ptr(h), ptr(nf)))
        return {"w": w, "h": h, "nfeatures": nf}

    def level_image(self, level: int, frame: int = 0, blurred: bool = False) -> np.ndarray:
        info = self.levels_info()
        out = np.empty((info["h"][level], info["w"][level]), np.uint8)
        check(lib().orbx_get_level(self._h, frame, level, int(blurred), ptr(out), out.strides[0]))
        return out

    @property
    def mvImagePyramid(self) -> list[np.ndarray]:
        """Pyramid of the last extraction (public member, include/ORBextractor.h:116)."""
        return [self.level_image(l) for l in range(self.nlevels)]

    def set_host_pyramid(self, enable: bool = True) -> None:
        """orbx_set_host_pyramid: later calls also leave their frame's pyramid in
        pinned host memory (copied beside FAST .. BRIEF inside the call)."""
        check(lib().orbx_set_host_pyramid(self._h, int(enable)))

    def host_pyramid(self) -> list[np.ndarray]:
        """The pinned host pyramid of the last call (orbx_get_host_pyramid), copied out."""
        L = self.nlevels
        ptrs = (C.c_void_p * L)()
        pitches = (C.c_size_t * L)()
        check(lib().orbx_get_host_pyramid(self._h, ptrs, pitches, L))
        info = self.levels_info()
        out = []
        for l in range(L):
            h, w, p = int(info["h"][l]), int(info["w"][l]), int(pitches[l])
            buf = (C.c_uint8 * (h * p)).from_address(ptrs[l])
            out.append(np.frombuffer(buf, np.uint8).reshape(h, p)[:, :w].copy())
        return out

    def fast_candidates(self, level: int, frame: int = 0) -> np.ndarray:
        """Stage probe: per-cell FAST+NMS output of the last extraction (pre-quadtree)."""
        cap = 1 << 20
        out = np.empty(cap, KP_DTYPE)
        n = C.c_int(0)
        check(lib().orbx_get_fast_candidates(self._h, frame, level, ptr(out), cap, C.byref(n)))
        return out[:n.value].copy()

    def stage_times(self) -> dict[str, float]:
        """Device ms per stage of the last extraction (needs ORBX_TIMING=1)."""
        ms = np.zeros(8, np.float32)
        names = (C.c_char_p * 8)()
        n = C.c_int(0)
        check(lib().orbx_get_stage_times(self._h, ptr(ms), names, 8, C.byref(n)))
        return {names[i].decode(): float(ms[i]) for i in range(n.value)}

    def tie_stats(self, frame0: int = 0, nframes: int = 1) -> np.ndarray:
        """Quadtree tie-rule exposure of the last extraction (orbx_get_tie_stats):
        int array (nframes, nlevels, 3) of {events, group nodes, kept keypoints}."""
        out = np.zeros((nframes, self.nlevels, 3), np.int32)
        check(lib().orbx_get_tie_stats(self._h, frame0, nframes, ptr(out)))
        return out

    def quadtree_paths(self, frame0: int = 0, nframes: int = 1) -> np.ndarray:
        """DistributeOctTree implementation per (frame, level) of the last extraction
        (orbx_get_quadtree_paths): 1 = sorted-key path, 0 = legacy rounds."""
        out = np.zeros((nframes, self.nlevels), np.int32)
        check(lib().orbx_get_quadtree_paths(self._h, frame0, nframes, ptr(out)))
        return out

    def status(self, reset: bool = True) -> int:
        """Device status word of the handle's kernels (orbx_get_status); 0 = ok."""
        st = C.c_int(0)
        check(lib().orbx_get_status(self._h, int(reset), C.byref(st)))
        return st.value


def brief_pattern(pattern: str = "fork") -> np.ndarray:
    """The rBRIEF test table the kernels use (orbx_get_pattern), 1024 ints in the
    reference's bit_pattern_31_ order (src/ORBextractor.cc:236-494). Host only."""
    out = np.zeros(1024, np.int32)
    check(lib().orbx_get_pattern(PATTERNS[pattern], ptr(out)))
    return out
