"""ORBVocabulary — host-side mirror of ORB_SLAM2::ORBVocabulary over liborbx.

ORBVocabulary is DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>
(include/ORBVocabulary.h:30). The parts on the hot path are mirrored:

    voc = ORBVocabulary()
    voc.loadFromTextFile("ORBvoc.txt")                  # System.cc vocabulary load
    bow, fv = voc.transform(descriptors, 4)             # Frame::ComputeBoW (src/Frame.cc:394-401)
    ComputeBoW(F, voc)                                  # fills F.mBowVec / F.mFeatVec

The tree lives on the GPU and the transform runs in the HIP kernels of
liborbx.so (orbx_vocab.hip); there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib, ptr


class ORBVocabulary:
    def __init__(self, *, device: int = 0):
        self.device = device
        self._h = C.c_void_p(0)

    # ---------------------------------------------------------- construction
    def loadFromTextFile(self, path: str) -> bool:
        """TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1338-1418)."""
        self.close()
        check(lib().orbv_load_text(path.encode(), self.device, C.byref(self._h)), vocabulary=True)
        return True

    @classmethod
    def from_arrays(cls, voc: dict, *, device: int = 0) -> "ORBVocabulary":
        """Node arrays in file order (see synth.synthetic_vocabulary)."""
        v = cls(device=device)
        parent = np.ascontiguousarray(voc["parent"], np.int32)
        leaf = np.ascontiguousarray(voc["leaf"], np.uint8)
        desc = np.ascontiguousarray(voc["desc"], np.uint8)
        weight = np.ascontiguousarray(voc["weight"], np.float64)
        check(lib().orbv_create(int(voc["k"]), int(voc["L"]), int(voc["scoring"]), int(voc["weighting"]),
                                len(parent), ptr(parent), ptr(leaf), ptr(desc), ptr(weight), device,
                                C.byref(v._h)), vocabulary=True)
        return v

    def close(self):
        if self._h and self._h.value:
            lib().orbv_destroy(self._h)
            self._h = C.c_void_p(0)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def _info(self):
        v = [C.c_int(0) for _ in range(6)]
        check(lib().orbv_info(self._h, *[C.byref(x) for x in v]), vocabulary=True)
        return [x.value for x in v]

    def getBranchingFactor(self) -> int:
        return self._info()[0]

    def getDepthLevels(self) -> int:
        return self._info()[1]

    def size(self) -> int:
        """Number of words."""
        return self._info()[5]

    def empty(self) -> bool:
        return self.size() == 0

    # ---------------------------------------------------------- transform
    def transform_arrays(self, descriptors: np.ndarray, levelsup: int = 4) -> dict:
        """transform(features, BowVector, FeatureVector, levelsup) as arrays: bow_words,
        bow_values (ascending words), fv_nodes, fv_off, fv_idx (CSR), and the
        per-feature word / node / weight."""
        d = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        n = len(d)
        m = max(n, 1)
        bw = np.zeros(m, np.uint32); bv = np.zeros(m, np.float64)
        fn = np.zeros(m, np.uint32); fo = np.zeros(m + 1, np.int32); fi = np.zeros(m, np.int32)
        wid = np.zeros(m, np.uint32); nid = np.zeros(m, np.uint32); wt = np.zeros(m, np.float64)
        nb, nf = C.c_int(0), C.c_int(0)
        check(lib().orbv_transform(self._h, ptr(d), n, levelsup, ptr(bw), ptr(bv), C.byref(nb), ptr(fn), ptr(fo),
                                   ptr(fi), C.byref(nf), ptr(wid), ptr(nid), ptr(wt)), vocabulary=True)
        b, f = nb.value, nf.value
        return dict(bow_words=bw[:b].copy(), bow_values=bv[:b].copy(), fv_nodes=fn[:f].copy(),
                    fv_off=fo[:f + 1].copy(), fv_idx=fi[:fo[f]].copy(), word=wid[:n].copy(), nid=nid[:n].copy(),
                    weight=wt[:n].copy())

    def transform(self, descriptors: np.ndarray, levelsup: int = 4):
        """Returns (BowVector {WordId: value}, FeatureVector {NodeId: [feature indices]})."""
        r = self.transform_arrays(descriptors, levelsup)
        bow = {int(w): float(v) for w, v in zip(r["bow_words"], r["bow_values"])}
        fv = {int(nd): r["fv_idx"][r["fv_off"][k]:r["fv_off"][k + 1]].tolist()
              for k, nd in enumerate(r["fv_nodes"])}
        return bow, fv


def ComputeBoW(F, voc: ORBVocabulary, levelsup: int = 4) -> None:
    """Frame::ComputeBoW (src/Frame.cc:394-401): mBowVec / mFeatVec of the frame's
    descriptors, computed once."""
    if getattr(F, "mBowVec", None):
        return
    F.mBowVec, F.mFeatVec = voc.transform(F.mDescriptors, levelsup)
