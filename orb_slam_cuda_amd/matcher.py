"""ORBmatcher — host-side mirror of ORB_SLAM2::ORBmatcher over liborbx.

Mirrors include/ORBmatcher.h:37-102 for the hot-path searches:

    m = ORBmatcher(nnratio=0.9, checkOri=True)
    nmatches = m.SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
    nmatches = m.SearchByBoW(pKF, F, vpMapPointMatches)          # KF - Frame
    nmatches = m.SearchByBoW(pKF1, pKF2, vpMatches12)            # KF - KF
    ORBmatcher.DescriptorDistance(a, b)

`Frame` / `KeyFrame` here are plain containers of the fields these searches
read (mvKeysUn, mDescriptors, the grid bounds, mFeatVec, MapPoint validity);
MapPoint pointers are represented by the index of the matched keypoint.
All searches run in the HIP kernels of liborbx.so.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from ._lib import KP_DTYPE, MAP_POINT_PROJ_DTYPE, FeatureVectorC, GridBounds, check, lib, ptr


@dataclass
class Frame:
    """The Frame fields read by SearchForInitialization / SearchByBoW."""
    mvKeysUn: np.ndarray                   # KP_DTYPE
    mDescriptors: np.ndarray               # (N, 32) uint8
    mnMinX: float = 0.0                    # image bounds (src/Frame.cc:445-461)
    mnMaxX: float = 0.0
    mnMinY: float = 0.0
    mnMaxY: float = 0.0
    mFeatVec: dict | None = None           # DBoW2::FeatureVector {NodeId: [feature idx]}
    mBowVec: dict | None = None            # DBoW2::BowVector {WordId: value}
    # stereo (Frame's stereo constructor, src/Frame.cc:43-101)
    mvKeysRight: np.ndarray | None = None  # KP_DTYPE
    mDescriptorsRight: np.ndarray | None = None
    mb: float = 0.0                        # baseline (m)
    mbf: float = 0.0                       # baseline x fx
    mvuRight: np.ndarray | None = None     # (N,) float32, -1 = no stereo match
    mvDepth: np.ndarray | None = None
    mvScaleFactors: np.ndarray | None = None  # (nlevels,) float32 (ORBextractor::GetScaleFactors)
    mvpMapPoints: np.ndarray | None = None    # (N,) int: map point index, -1 = NULL

    @property
    def N(self) -> int:
        return len(self.mvKeysUn)

    @property
    def mvKeys(self) -> np.ndarray:
        return self.mvKeysUn

    @classmethod
    def from_extraction(cls, kps, desc, width, height, featvec=None):
        # no distortion: mvKeysUn == mvKeys and bounds = image rectangle (src/Frame.cc:458-461)
        return cls(kps, desc, 0.0, float(width), 0.0, float(height), featvec)


def ComputeStereoMatches(F: Frame, extractorLeft, extractorRight, matcher: "ORBmatcher") -> int:
    """Frame::ComputeStereoMatches (src/Frame.cc:465-639): fills F.mvuRight / F.mvDepth from
    F.mvKeys/mDescriptors (left) and F.mvKeysRight/mDescriptorsRight, refining with the
    mvImagePyramid of the two extractors' last extraction (frame 0 of each). Returns the
    number of stereo matches kept after the median-SAD rejection."""
    kpL = np.ascontiguousarray(F.mvKeysUn, KP_DTYPE)
    kpR = np.ascontiguousarray(F.mvKeysRight, KP_DTYPE)
    dL = np.ascontiguousarray(F.mDescriptors, np.uint8)
    dR = np.ascontiguousarray(F.mDescriptorsRight, np.uint8)
    uR = np.full(len(kpL), -1.0, np.float32)
    dep = np.full(len(kpL), -1.0, np.float32)
    kept = C.c_int(0)
    check(lib().orbm_compute_stereo_matches(
        matcher.handle, extractorLeft.handle, extractorRight.handle, ptr(kpL), ptr(dL), len(kpL),
        ptr(kpR), ptr(dR), len(kpR), C.c_float(F.mb), C.c_float(F.mbf), ptr(uR), ptr(dep),
        C.byref(kept)), matcher=True)
    F.mvuRight, F.mvDepth = uR, dep
    return kept.value


@dataclass
class KeyFrame:
    mvKeysUn: np.ndarray
    mDescriptors: np.ndarray
    mvpMapPoints: np.ndarray               # bool/uint8: MapPoint present and !isBad()
    mFeatVec: dict = field(default_factory=dict)

    @property
    def N(self) -> int:
        return len(self.mvKeysUn)


def feature_vector_csr(fv: dict):
    nodes = np.array(sorted(fv), dtype=np.uint32)
    off = np.zeros(len(nodes) + 1, np.int32)
    idx = []
    for k, n in enumerate(nodes):
        v = list(fv[int(n)])
        idx.extend(v)
        off[k + 1] = off[k] + len(v)
    return nodes, off, np.asarray(idx, np.int32)


def _fvc(csr):
    nodes, off, idx = csr
    return FeatureVectorC(nodes.ctypes.data, off.ctypes.data, idx.ctypes.data if len(idx) else 0, len(nodes))


class ORBmatcher:
    TH_HIGH = 100   # src/ORBmatcher.cc:37
    TH_LOW = 50     # :38
    HISTO_LENGTH = 30  # :39

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, *, device: int = 0,
                 max_pairs: int = 1, max_kps: int = 4096):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        self.device = device
        self._h = C.c_void_p(0)
        check(lib().orbm_create(device, max_pairs, max_kps, C.byref(self._h)), matcher=True)
        self.max_kps = max_kps

    def close(self):
        if self._h and self._h.value:
            lib().orbm_destroy(self._h)
            self._h = C.c_void_p(0)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    @staticmethod
    def DescriptorDistance(a: np.ndarray, b: np.ndarray) -> int:
        a = np.ascontiguousarray(a, np.uint8).reshape(32)
        b = np.ascontiguousarray(b, np.uint8).reshape(32)
        return lib().orbm_descriptor_distance(ptr(a), ptr(b))

    def SearchForInitialization(self, F1: Frame, F2: Frame, vbPrevMatched: np.ndarray,
                                vnMatches12: list | None = None, windowSize: int = 10) -> int:
        """vbPrevMatched: (N1, 2) float32, updated in place; vnMatches12 (list) is filled."""
        kp1 = np.ascontiguousarray(F1.mvKeysUn, KP_DTYPE)
        kp2 = np.ascontiguousarray(F2.mvKeysUn, KP_DTYPE)
        d1 = np.ascontiguousarray(F1.mDescriptors, np.uint8)
        d2 = np.ascontiguousarray(F2.mDescriptors, np.uint8)
        prev = np.ascontiguousarray(vbPrevMatched, np.float32)
        assert prev.shape == (len(kp1), 2)
        m12 = np.full(len(kp1), -1, np.int32)
        nm = C.c_int(0)
        b = GridBounds(F2.mnMinX, F2.mnMaxX, F2.mnMinY, F2.mnMaxY)
        check(lib().orbm_search_for_initialization(
            self._h, ptr(kp1), ptr(d1), len(kp1), ptr(kp2), ptr(d2), len(kp2), b, ptr(prev),
            int(windowSize), C.c_float(self.mfNNratio), int(self.mbCheckOrientation), ptr(m12),
            C.byref(nm)), matcher=True)
        if prev is not vbPrevMatched:
            vbPrevMatched[...] = prev
        if vnMatches12 is not None:
            vnMatches12[:] = m12.tolist()
        self.last_matches12 = m12
        return nm.value

    def SearchByProjection(self, F: Frame, mps: np.ndarray, mp_desc: np.ndarray, th: float = 3.0,
                           blocked: np.ndarray | None = None) -> int:
        """SearchByProjection(Frame&, const vector<MapPoint*>&, th) (src/ORBmatcher.cc:45-118).
        mps: MAP_POINT_PROJ_DTYPE per map point (Frame::isInFrustum's mTrackProj*, view cos,
        predicted level, in-view and Observations() > 0 flags), mp_desc their descriptors.
        blocked[idx]: keypoint idx already holds a map point with observations (default:
        F.mvpMapPoints >= 0). Assigned keypoints get the map point's index in F.mvpMapPoints."""
        kps = np.ascontiguousarray(F.mvKeysUn, KP_DTYPE)
        d = np.ascontiguousarray(F.mDescriptors, np.uint8)
        n = len(kps)
        if F.mvpMapPoints is None:
            F.mvpMapPoints = np.full(n, -1, np.int32)
        if blocked is None:
            blocked = F.mvpMapPoints >= 0
        bl = np.ascontiguousarray(blocked, np.uint8)
        ur = None if F.mvuRight is None else np.ascontiguousarray(F.mvuRight, np.float32)
        sc = np.ascontiguousarray(F.mvScaleFactors, np.float32)
        mp = np.ascontiguousarray(mps, MAP_POINT_PROJ_DTYPE)
        md = np.ascontiguousarray(mp_desc, np.uint8)
        out = np.full(max(n, 1), -1, np.int32)
        nm = C.c_int(0)
        b = GridBounds(F.mnMinX, F.mnMaxX, F.mnMinY, F.mnMaxY)
        check(lib().orbm_search_by_projection(self._h, ptr(kps), ptr(d), n, ptr(ur), b, ptr(sc), len(sc), ptr(bl),
                                              ptr(mp), ptr(md), len(mp), C.c_float(th), C.c_float(self.mfNNratio),
                                              ptr(out), C.byref(nm)), matcher=True)
        hit = out[:n] >= 0
        F.mvpMapPoints[hit] = out[:n][hit]
        self.last_projection = out[:n].copy()
        return nm.value

    def SearchByBoW(self, A: KeyFrame, B, out: list | None = None) -> int:
        """KF-Frame (B is a Frame) or KF-KF (B is a KeyFrame). Fills `out` with matched
        indices (-1 = NULL MapPoint) like vpMapPointMatches / vpMatches12."""
        kf_vs_kf = isinstance(B, KeyFrame)
        fa = feature_vector_csr(A.mFeatVec)
        fb = feature_vector_csr(B.mFeatVec or {})
        dA = np.ascontiguousarray(A.mDescriptors, np.uint8)
        dB = np.ascontiguousarray(B.mDescriptors, np.uint8)
        aA = np.ascontiguousarray(A.mvKeysUn["angle"], np.float32)
        aB = np.ascontiguousarray((B.mvKeysUn if kf_vs_kf else B.mvKeys)["angle"], np.float32)
        mA = np.ascontiguousarray(A.mvpMapPoints, np.uint8)
        mB = np.ascontiguousarray(B.mvpMapPoints, np.uint8) if kf_vs_kf else None
        res = np.full(len(dA) if kf_vs_kf else len(dB), -1, np.int32)
        nm = C.c_int(0)
        check(lib().orbm_search_by_bow(
            self._h, ptr(dA), ptr(aA), ptr(mA), len(dA), _fvc(fa), ptr(dB), ptr(aB), ptr(mB), len(dB),
            _fvc(fb), C.c_float(self.mfNNratio), int(self.mbCheckOrientation), int(kf_vs_kf), ptr(res),
            C.byref(nm)), matcher=True)
        if out is not None:
            out[:] = res.tolist()
        self.last_matches = res
        return nm.value
