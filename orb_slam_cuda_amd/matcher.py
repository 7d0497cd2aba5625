"""ORBmatcher — host-side mirror of ORB_SLAM2::ORBmatcher over liborbx.

Mirrors include/ORBmatcher.h:37-102 for the hot-path searches:

    m = ORBmatcher(nnratio=0.9, checkOri=True)
    nmatches = m.SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
    nmatches = m.SearchByBoW(pKF, F, vpMapPointMatches)          # KF - Frame
    nmatches = m.SearchByBoW(pKF1, pKF2, vpMatches12)            # KF - KF
    nmatches = m.SearchByProjection(F, mps, mp_desc, th)         # local map (Frame::isInFrustum records)
    nmatches = m.SearchByProjection(CurrentFrame, LastFrame, th, bMono)
    nmatches = m.SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
    nmatches = m.SearchByProjection(pKF, Scw, vpPoints, vpMatched, th)
    nmatches = m.SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo)
    nfused   = m.Fuse(pKF, vpMapPoints, th)                      # matching part, see Fuse()
    nfused   = m.Fuse(pKF, Scw, vpPoints, th, vpReplacePoint)
    nfound   = m.SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)
    ORBmatcher.DescriptorDistance(a, b)

`Frame` / `KeyFrame` here are plain containers of the fields these searches
read (mvKeysUn, mDescriptors, the grid bounds, camera and pose, mFeatVec,
MapPoint links). MapPoint pointers are row indices into a `MapPoints` table
(the Map), -1 standing for NULL.
All searches run in the HIP kernels of liborbx.so.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import (KP_DTYPE, MAP_POINT_PROJ_DTYPE, MAP_POINT_WORLD_DTYPE, FeatureVectorC, GridBounds, camera, check,
                   lib, ptr)


@dataclass
class MapPoints:
    """The MapPoint fields the searches read, one row per MapPoint (a pointer is a row index):
    GetWorldPos, GetNormal, mfMinDistance / mfMaxDistance, GetDescriptor, Observations(), isBad()."""
    pos: np.ndarray                        # (M, 3) float32
    descriptors: np.ndarray                # (M, 32) uint8
    normal: np.ndarray | None = None       # (M, 3) float32
    min_distance: np.ndarray | None = None  # (M,) float32
    max_distance: np.ndarray | None = None  # (M,) float32
    nobs: np.ndarray | None = None         # (M,) int, default 1
    bad: np.ndarray | None = None          # (M,) bool, default False

    def __len__(self):
        return len(self.pos)

    def records(self, idx, angle=None, octave=None, valid=None):
        """orbm_map_point_world records + descriptors for pointers idx (-1 = NULL -> not valid)."""
        idx = np.asarray(idx, np.int64)
        ok = idx >= 0
        j = np.where(ok, idx, 0)
        M = len(self)
        rec = np.zeros(len(idx), MAP_POINT_WORLD_DTYPE)
        if M == 0:
            return rec, np.zeros((len(idx), 32), np.uint8)
        rec["pos"] = np.asarray(self.pos, np.float32)[j]
        if self.normal is not None:
            rec["normal"] = np.asarray(self.normal, np.float32)[j]
        if self.min_distance is not None:
            rec["min_distance"] = np.asarray(self.min_distance, np.float32)[j]
        if self.max_distance is not None:
            rec["max_distance"] = np.asarray(self.max_distance, np.float32)[j]
        if angle is not None:
            rec["angle"] = angle
        if octave is not None:
            rec["octave"] = octave
        bad = np.zeros(M, bool) if self.bad is None else np.asarray(self.bad, bool)
        nobs = np.ones(M, np.int64) if self.nobs is None else np.asarray(self.nobs)
        rec["valid"] = ok & (True if valid is None else np.asarray(valid, bool))
        rec["obs_positive"] = ok & (nobs[j] > 0)
        return rec, np.ascontiguousarray(np.asarray(self.descriptors, np.uint8)[j])

    def bad_of(self, idx):
        idx = np.asarray(idx, np.int64)
        if self.bad is None:
            return np.zeros(len(idx), bool)
        return np.asarray(self.bad, bool)[np.where(idx >= 0, idx, 0)] & (idx >= 0)

    def obs_of(self, idx):
        idx = np.asarray(idx, np.int64)
        nobs = np.ones(len(self), np.int64) if self.nobs is None else np.asarray(self.nobs)
        return (idx >= 0) & (nobs[np.where(idx >= 0, idx, 0)] > 0)


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
    # camera and pose (SearchByProjection overloads that project world points)
    fx: float = 0.0
    fy: float = 0.0
    cx: float = 0.0
    cy: float = 0.0
    mTcw: np.ndarray | None = None         # (3, 4) or (4, 4) float32
    mvbOutlier: np.ndarray | None = None   # (N,) bool
    mfScaleFactor: float = 1.2
    mpMap: "MapPoints | None" = None

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


def ComputeStereoMatchesLast(F: Frame, extractorLeft, extractorRight, matcher: "ORBmatcher") -> int:
    """Frame::ComputeStereoMatches as the stereo constructor runs it, right after its two
    extractions (src/Frame.cc:77-89): the keypoints and descriptors are the ones the two
    extractors' last calls left on the device (orbm_compute_stereo_matches_last); F.mvKeys
    must be the left call's output. Fills F.mvuRight / F.mvDepth, returns the kept count."""
    n = len(F.mvKeysUn)
    uR = np.full(n, -1.0, np.float32)
    dep = np.full(n, -1.0, np.float32)
    kept = C.c_int(0)
    check(lib().orbm_compute_stereo_matches_last(
        matcher.handle, extractorLeft.handle, extractorRight.handle, C.c_float(F.mb), C.c_float(F.mbf),
        ptr(uR), ptr(dep), n, C.byref(kept)), matcher=True)
    F.mvuRight, F.mvDepth = uR, dep
    return kept.value


def ExtractStereo(extractorLeft, extractorRight, imLeft, imRight, matcher: "ORBmatcher", mb: float,
                  mbf: float):
    """The stereo Frame constructor's extraction and matching steps (src/Frame.cc:77-89:
    ExtractORB on threadLeft / threadRight, then ComputeStereoMatches) with one device round
    trip (orbm_stereo_frame). Returns (keysLeft, descLeft, keysRight, descRight, mvuRight,
    mvDepth, kept), equal to the two extractor calls followed by ComputeStereoMatchesLast."""
    imgs = []
    for im in (imLeft, imRight):
        im = np.asarray(im)
        if im.size and (im.dtype != np.uint8 or im.ndim != 2):
            raise _lib.OrbxError(_lib.ORBX_EINVAL, "image must be CV_8UC1 (2-D uint8)")
        imgs.append(np.ascontiguousarray(im) if im.size and im.strides[1] != 1 else im)
    L, R = imgs
    if L.size == 0 or R.size == 0 or L.shape != R.shape:
        kL, dL = extractorLeft(L)
        kR, dR = extractorRight(R)
        F = Frame.from_extraction(kL, dL, 0, 0)
        F.mb, F.mbf = mb, mbf
        kept = ComputeStereoMatchesLast(F, extractorLeft, extractorRight, matcher)
        return kL, dL, kR, dR, F.mvuRight, F.mvDepth, kept
    capL, capR = extractorLeft._begin(L), extractorRight._begin(R)
    kL, kR = np.empty(capL, KP_DTYPE), np.empty(capR, KP_DTYPE)
    dL, dR = np.empty((capL, 32), np.uint8), np.empty((capR, 32), np.uint8)
    uR = np.full(capL, -1.0, np.float32)
    dep = np.full(capL, -1.0, np.float32)
    nL, nR, kept = C.c_int(0), C.c_int(0), C.c_int(0)
    check(lib().orbm_stereo_frame(
        matcher.handle, extractorLeft.handle, extractorRight.handle, ptr(L), L.strides[0], ptr(R), R.strides[0],
        L.shape[1], L.shape[0], C.c_float(mb), C.c_float(mbf), ptr(kL), capL, ptr(dL), C.byref(nL), ptr(kR),
        capR, ptr(dR), C.byref(nR), ptr(uR), ptr(dep), C.byref(kept)), matcher=True)
    n, m = nL.value, nR.value
    return (kL[:n].copy(), dL[:n].copy(), kR[:m].copy(), dR[:m].copy(), uR[:n].copy(), dep[:n].copy(),
            kept.value)


@dataclass
class KeyFrame:
    mvKeysUn: np.ndarray
    mDescriptors: np.ndarray
    mvpMapPoints: np.ndarray               # bool/uint8 mask (MapPoint present and !isBad()) or int pointers (-1 = NULL)
    mFeatVec: dict = field(default_factory=dict)
    mnMinX: float = 0.0
    mnMaxX: float = 0.0
    mnMinY: float = 0.0
    mnMaxY: float = 0.0
    fx: float = 0.0
    fy: float = 0.0
    cx: float = 0.0
    cy: float = 0.0
    mvScaleFactors: np.ndarray | None = None
    mfScaleFactor: float = 1.2
    mpMap: "MapPoints | None" = None
    mTcw: np.ndarray | None = None         # (3, 4) or (4, 4) float32
    mvuRight: np.ndarray | None = None     # (N,) float32, -1 = monocular
    mbf: float = 0.0
    mvLevelSigma2: np.ndarray | None = None
    mvInvLevelSigma2: np.ndarray | None = None

    def GetCameraCenter(self) -> np.ndarray:
        """Ow = -Rcw^T tcw (KeyFrame::SetPose, src/KeyFrame.cc:77-92)."""
        T = np.asarray(self.mTcw, np.float64)
        return (-T[:3, :3].T @ T[:3, 3]).astype(np.float32)

    @property
    def N(self) -> int:
        return len(self.mvKeysUn)


def _mp_mask(a) -> np.ndarray:
    """MapPoint presence from a bool/uint8 mask or an int pointer array (-1 = NULL)."""
    a = np.asarray(a)
    return (a != 0) if a.dtype in (np.bool_, np.uint8) else (a >= 0)


def _grid(F) -> GridBounds:
    return GridBounds(F.mnMinX, F.mnMaxX, F.mnMinY, F.mnMaxY)


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

    def status(self, reset: bool = True) -> int:
        """Device status word of the matcher's batched kernels (orbm_get_status); 0 = ok."""
        st = C.c_int(0)
        check(lib().orbm_get_status(self._h, int(reset), C.byref(st)), matcher=True)
        return st.value

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

    def SearchByProjection(self, a, b, *args, **kw) -> int:
        """The four SearchByProjection overloads (include/ORBmatcher.h:48-60), by argument types:
        (Frame, records, descriptors, th=3)            local map       src/ORBmatcher.cc:45-118
        (Frame CurrentFrame, Frame LastFrame, th, bMono)  motion model  :1328-1470
        (Frame CurrentFrame, KeyFrame pKF, sAlreadyFound, th, ORBdist)  relocalization :1472-1599
        (KeyFrame pKF, Scw, vpPoints, vpMatched, th)  loop closing     :290-403"""
        if isinstance(a, KeyFrame):
            return self._search_sim3(a, b, *args, **kw)
        if isinstance(b, Frame):
            return self._search_last_frame(a, b, *args, **kw)
        if isinstance(b, KeyFrame):
            return self._search_keyframe(a, b, *args, **kw)
        return self._search_local_map(a, b, *args, **kw)

    def SearchForTriangulation(self, pKF1: KeyFrame, pKF2: KeyFrame, F12, vMatchedPairs: list | None,
                               bOnlyStereo: bool) -> int:
        """SearchForTriangulation (src/ORBmatcher.cc:657-823): vMatchedPairs <- [(idx1, idx2)] in idx1 order."""
        def side(K):
            return (np.ascontiguousarray(K.mvKeysUn, KP_DTYPE), np.ascontiguousarray(K.mDescriptors, np.uint8),
                    np.ascontiguousarray(np.full(K.N, -1, np.float32) if K.mvuRight is None else K.mvuRight,
                                         np.float32),
                    np.ascontiguousarray(_mp_mask(K.mvpMapPoints), np.uint8), feature_vector_csr(K.mFeatVec))
        k1, d1, u1, h1, fv1 = side(pKF1)
        k2, d2, u2, h2, fv2 = side(pKF2)
        cw1 = np.ascontiguousarray(pKF1.GetCameraCenter(), np.float32)
        T2 = np.ascontiguousarray(np.asarray(pKF2.mTcw, np.float32)[:3], np.float32)
        cam2 = np.array([pKF2.fx, pKF2.fy, pKF2.cx, pKF2.cy], np.float32)
        sc2 = np.ascontiguousarray(pKF2.mvScaleFactors, np.float32)
        sg2 = np.ascontiguousarray(pKF2.mvLevelSigma2, np.float32)
        F = np.ascontiguousarray(F12, np.float32).reshape(9)
        out = np.full(max(len(k1), 1), -1, np.int32)
        nm = C.c_int(0)
        check(lib().orbm_search_for_triangulation(
            self._h, ptr(k1), ptr(d1), ptr(u1), ptr(h1), len(k1), _fvc(fv1), ptr(k2), ptr(d2), ptr(u2), ptr(h2),
            len(k2), _fvc(fv2), ptr(cw1), ptr(T2), ptr(cam2), ptr(sc2), ptr(sg2), len(sc2), ptr(F),
            int(bool(bOnlyStereo)), int(self.mbCheckOrientation), ptr(out), C.byref(nm)), matcher=True)
        m12 = out[:len(k1)]
        if vMatchedPairs is not None:
            vMatchedPairs[:] = [(int(i), int(j)) for i, j in enumerate(m12) if j >= 0]
        self.last_matches = m12.copy()
        return nm.value

    def Fuse(self, pKF: KeyFrame, *args) -> int:
        """Fuse(pKF, vpMapPoints, th=3.0) (src/ORBmatcher.cc:825-975) or
        Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (:977-1100).

        The GPU computes every point's match against pKF; the in-order tail of the reference is
        applied here on the pointer arrays: a point matched to a keypoint without a MapPoint is
        added (pKF.mvpMapPoints[idx] = point, so later points see it); otherwise the Scw overload
        records vpReplacePoint[i] = the keypoint's MapPoint (if not bad) and the first overload
        records the (point, keypoint MapPoint) pair in self.last_fuse_replace (MapPoint::Replace
        itself belongs to the Map, outside this matcher). self.last_fuse = per-point keypoints."""
        mp = pKF.mpMap
        kps = np.ascontiguousarray(pKF.mvKeysUn, KP_DTYPE)
        d = np.ascontiguousarray(pKF.mDescriptors, np.uint8)
        n = len(kps)
        sc = np.ascontiguousarray(pKF.mvScaleFactors, np.float32)
        kmp = np.asarray(pKF.mvpMapPoints, np.int64).copy()
        sim3 = len(args) >= 3
        if sim3:
            Scw, vpPoints, th, vpReplacePoint = args[0], args[1], args[2], (args[3] if len(args) > 3 else None)
            pts = np.asarray(vpPoints, np.int64)
            found = np.isin(pts, kmp[kmp >= 0])  # spAlreadyFound = pKF->GetMapPoints()
            rec, md = mp.records(pts, None, None, ~mp.bad_of(pts) & ~found)
            cam = camera(pKF.fx, pKF.fy, pKF.cx, pKF.cy, 0.0, 0.0, Scw)
        else:
            vpMapPoints, th = args[0], (args[1] if len(args) > 1 else 3.0)
            pts = np.asarray(vpMapPoints, np.int64)
            inkf = np.isin(pts, kmp[kmp >= 0])  # IsInKeyFrame(pKF)
            rec, md = mp.records(pts, None, None, ~mp.bad_of(pts) & ~inkf)
            cam = camera(pKF.fx, pKF.fy, pKF.cx, pKF.cy, 0.0, pKF.mbf, pKF.mTcw)
        out = np.full(max(len(pts), 1), -1, np.int32)
        nm = C.c_int(0)
        if sim3:
            check(lib().orbm_fuse_sim3(self._h, ptr(kps), ptr(d), n, _grid(pKF), ptr(sc), len(sc),
                                       C.c_float(pKF.mfScaleFactor), C.byref(cam), ptr(rec), ptr(md), len(rec),
                                       C.c_float(th), ptr(out), C.byref(nm)), matcher=True)
        else:
            ur = None if pKF.mvuRight is None else np.ascontiguousarray(pKF.mvuRight, np.float32)
            isg = np.ascontiguousarray(pKF.mvInvLevelSigma2, np.float32)
            check(lib().orbm_fuse(self._h, ptr(kps), ptr(d), n, ptr(ur), _grid(pKF), ptr(sc), ptr(isg), len(sc),
                                  C.c_float(pKF.mfScaleFactor), C.byref(cam), ptr(rec), ptr(md), len(rec),
                                  C.c_float(th), ptr(out), C.byref(nm)), matcher=True)
        o = out[:len(pts)]
        self.last_fuse = o.copy()
        replace = []
        for i in np.nonzero(o >= 0)[0]:  # the reference's in-order tail (:932-957, :1083-1097)
            idx = int(o[i])
            cur = int(kmp[idx])
            if cur >= 0:
                if not mp.bad_of([cur])[0]:
                    if sim3 and vpReplacePoint is not None:
                        vpReplacePoint[i] = cur
                    replace.append((int(pts[i]), cur))
            else:
                kmp[idx] = pts[i]
        if isinstance(pKF.mvpMapPoints, np.ndarray) and pKF.mvpMapPoints.dtype.kind == "i":
            pKF.mvpMapPoints[:] = kmp
        self.last_fuse_replace = replace
        return nm.value

    def SearchBySim3(self, pKF1: KeyFrame, pKF2: KeyFrame, vpMatches12, s12: float, R12, t12, th: float) -> int:
        """SearchBySim3 (src/ORBmatcher.cc:1102-1326): vpMatches12 (pKF1.N pointers, -1 = NULL) gains the
        new mutual matches."""
        mp = pKF1.mpMap
        m1 = np.asarray(pKF1.mvpMapPoints, np.int64)
        m2 = np.asarray(pKF2.mvpMapPoints, np.int64)
        vm = np.asarray(vpMatches12, np.int64)
        already1 = vm >= 0
        already2 = np.isin(m2, vm[vm >= 0]) & (m2 >= 0)  # pMP->GetIndexInKeyFrame(pKF2)
        r1, q1 = mp.records(m1, None, None, ~already1 & ~mp.bad_of(m1))
        r2, q2 = mp.records(m2, None, None, ~already2 & ~mp.bad_of(m2))
        k1 = np.ascontiguousarray(pKF1.mvKeysUn, KP_DTYPE)
        k2 = np.ascontiguousarray(pKF2.mvKeysUn, KP_DTYPE)
        d1 = np.ascontiguousarray(pKF1.mDescriptors, np.uint8)
        d2 = np.ascontiguousarray(pKF2.mDescriptors, np.uint8)
        T1 = np.ascontiguousarray(np.asarray(pKF1.mTcw, np.float32)[:3], np.float32)
        T2 = np.ascontiguousarray(np.asarray(pKF2.mTcw, np.float32)[:3], np.float32)
        sc = np.ascontiguousarray(pKF2.mvScaleFactors, np.float32)
        cam1 = camera(pKF1.fx, pKF1.fy, pKF1.cx, pKF1.cy, 0.0, 0.0, T1)
        R = np.ascontiguousarray(R12, np.float32).reshape(9)
        t = np.ascontiguousarray(t12, np.float32).reshape(3)
        out = np.full(max(len(k1), 1), -1, np.int32)
        nf = C.c_int(0)
        check(lib().orbm_search_by_sim3(
            self._h, ptr(k1), ptr(d1), len(k1), _grid(pKF1), ptr(T1), ptr(r1), ptr(q1), ptr(k2), ptr(d2), len(k2),
            _grid(pKF2), ptr(T2), ptr(r2), ptr(q2), ptr(sc), len(sc), C.c_float(pKF2.mfScaleFactor), C.byref(cam1),
            C.c_float(s12), ptr(R), ptr(t), C.c_float(th), ptr(out), C.byref(nf)), matcher=True)
        o = out[:len(k1)]
        for i1 in np.nonzero(o >= 0)[0]:
            vpMatches12[i1] = int(m2[o[i1]])
        self.last_matches = o.copy()
        return nf.value

    def _search_last_frame(self, CurrentFrame: Frame, LastFrame: Frame, th: float, bMono: bool) -> int:
        """SearchByProjection(Frame&, const Frame&, th, bMono): map points of LastFrame (not outliers)
        projected with CurrentFrame.mTcw; stores pointers into CurrentFrame.mvpMapPoints."""
        F, L, mp = CurrentFrame, LastFrame, CurrentFrame.mpMap
        kps = np.ascontiguousarray(F.mvKeysUn, KP_DTYPE)
        d = np.ascontiguousarray(F.mDescriptors, np.uint8)
        n = len(kps)
        if F.mvpMapPoints is None:
            F.mvpMapPoints = np.full(n, -1, np.int32)
        lmp = np.asarray(L.mvpMapPoints, np.int64)
        outl = np.zeros(L.N, bool) if L.mvbOutlier is None else np.asarray(L.mvbOutlier, bool)
        rec, md = mp.records(lmp, L.mvKeysUn["angle"], L.mvKeys["octave"], ~outl)
        bl = np.ascontiguousarray(mp.obs_of(F.mvpMapPoints), np.uint8)
        ur = None if F.mvuRight is None else np.ascontiguousarray(F.mvuRight, np.float32)
        sc = np.ascontiguousarray(F.mvScaleFactors, np.float32)
        cam = camera(F.fx, F.fy, F.cx, F.cy, F.mb, F.mbf, F.mTcw)
        Tlw = np.ascontiguousarray(np.asarray(L.mTcw, np.float32)[:3], np.float32)
        out = np.full(max(n, 1), -1, np.int32)
        nm = C.c_int(0)
        check(lib().orbm_search_by_projection_last_frame(
            self._h, ptr(kps), ptr(d), n, ptr(ur), _grid(F), ptr(sc), len(sc), ptr(bl), C.byref(cam), ptr(Tlw),
            ptr(rec), ptr(md), len(rec), C.c_float(th), int(bool(bMono)), int(self.mbCheckOrientation), ptr(out),
            C.byref(nm)), matcher=True)
        o = out[:n]
        F.mvpMapPoints[o >= 0] = lmp[o[o >= 0]]
        F.mvpMapPoints[o == -2] = -1
        self.last_projection = o.copy()
        return nm.value

    def _search_keyframe(self, CurrentFrame: Frame, pKF: KeyFrame, sAlreadyFound, th: float, ORBdist: int) -> int:
        """SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist)."""
        F, mp = CurrentFrame, CurrentFrame.mpMap
        kps = np.ascontiguousarray(F.mvKeysUn, KP_DTYPE)
        d = np.ascontiguousarray(F.mDescriptors, np.uint8)
        n = len(kps)
        if F.mvpMapPoints is None:
            F.mvpMapPoints = np.full(n, -1, np.int32)
        kmp = np.asarray(pKF.mvpMapPoints, np.int64)  # pKF->GetMapPointMatches()
        found = np.isin(kmp, np.fromiter(sAlreadyFound, np.int64)) if len(sAlreadyFound) else np.zeros(len(kmp), bool)
        rec, md = mp.records(kmp, pKF.mvKeysUn["angle"], None, ~mp.bad_of(kmp) & ~found)
        hm = np.ascontiguousarray(np.asarray(F.mvpMapPoints) >= 0, np.uint8)
        sc = np.ascontiguousarray(F.mvScaleFactors, np.float32)
        cam = camera(F.fx, F.fy, F.cx, F.cy, F.mb, F.mbf, F.mTcw)
        out = np.full(max(n, 1), -1, np.int32)
        nm = C.c_int(0)
        check(lib().orbm_search_by_projection_keyframe(
            self._h, ptr(kps), ptr(d), n, _grid(F), ptr(sc), len(sc), C.c_float(F.mfScaleFactor), ptr(hm),
            C.byref(cam), ptr(rec), ptr(md), len(rec), C.c_float(th), int(ORBdist), int(self.mbCheckOrientation),
            ptr(out), C.byref(nm)), matcher=True)
        o = out[:n]
        F.mvpMapPoints[o >= 0] = kmp[o[o >= 0]]
        F.mvpMapPoints[o == -2] = -1
        self.last_projection = o.copy()
        return nm.value

    def _search_sim3(self, pKF: KeyFrame, Scw, vpPoints, vpMatched, th: int) -> int:
        """SearchByProjection(KeyFrame*, cv::Mat Scw, const vector<MapPoint*>&, vector<MapPoint*>&, th):
        vpMatched (pKF.N pointers, -1 = NULL) is updated in place."""
        mp = pKF.mpMap
        kps = np.ascontiguousarray(pKF.mvKeysUn, KP_DTYPE)
        d = np.ascontiguousarray(pKF.mDescriptors, np.uint8)
        n = len(kps)
        pts = np.asarray(vpPoints, np.int64)
        matched = np.asarray(vpMatched, np.int64)
        already = np.isin(pts, matched[matched >= 0])
        rec, md = mp.records(pts, None, None, ~mp.bad_of(pts) & ~already)
        mt = np.ascontiguousarray(np.where(matched >= 0, 0, -1), np.int32)
        sc = np.ascontiguousarray(pKF.mvScaleFactors, np.float32)
        cam = camera(pKF.fx, pKF.fy, pKF.cx, pKF.cy, 0.0, 0.0, Scw)
        out = np.full(max(n, 1), -1, np.int32)
        nm = C.c_int(0)
        check(lib().orbm_search_by_projection_sim3(
            self._h, ptr(kps), ptr(d), n, _grid(pKF), ptr(sc), len(sc), C.c_float(pKF.mfScaleFactor), C.byref(cam),
            ptr(rec), ptr(md), len(rec), int(th), ptr(mt), ptr(out), C.byref(nm)), matcher=True)
        o = out[:n]
        res = matched.copy()
        res[o >= 0] = pts[o[o >= 0]]
        vpMatched[:] = res.tolist() if isinstance(vpMatched, list) else res
        self.last_projection = o.copy()
        return nm.value

    def _search_local_map(self, F: Frame, mps: np.ndarray, mp_desc: np.ndarray, th: float = 3.0,
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
        mA = np.ascontiguousarray(_mp_mask(A.mvpMapPoints), np.uint8)
        mB = np.ascontiguousarray(_mp_mask(B.mvpMapPoints), np.uint8) if kf_vs_kf else None
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
