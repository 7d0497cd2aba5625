"""ctypes wrapper of the CPU ORACLE (oracle/liborb_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package. The oracle is the
checker: a CPU restatement of the reference path (see orb_oracle.h for the
per-function reference citations and the "parity unpinned" status).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liborb_oracle.so")

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KP_DTYPE.itemsize == 28


class OrcConfig(C.Structure):
    _fields_ = [("nfeatures", C.c_int), ("scale_factor", C.c_float), ("nlevels", C.c_int),
                ("ini_th_fast", C.c_int), ("min_th_fast", C.c_int), ("width", C.c_int),
                ("height", C.c_int), ("scale_mode", C.c_int), ("pattern_mode", C.c_int)]


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.orc_fast_atan2.restype = C.c_float
        _lib.orc_fast_atan2.argtypes = [C.c_float, C.c_float]
        _lib.orc_sincosf.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        _lib.orc_compute_stereo_matches.argtypes = [
            C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_float,
            C.c_float, C.c_void_p, C.c_void_p]
        _lib.orc_search_by_projection.argtypes = ([C.c_void_p] * 2 + [C.c_int, C.c_void_p] + [C.c_float] * 4
                                                  + [C.c_void_p] * 4 + [C.c_int, C.c_float, C.c_float]
                                                  + [C.c_void_p] * 2)
        _lib.orc_voc_load_text.argtypes = [C.c_char_p] + [C.c_void_p] * 5 + [C.c_int] + [C.c_void_p] * 4
        _lib.orc_voc_transform.argtypes = ([C.c_int] * 5 + [C.c_void_p] * 5 + [C.c_int, C.c_int]
                                           + [C.c_void_p] * 10)
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def config(nfeatures=2000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7, width=1241,
           height=376, scale_mode=0, pattern_mode=0) -> OrcConfig:
    return OrcConfig(nfeatures, scale_factor, nlevels, ini_th, min_th, width, height,
                     scale_mode, pattern_mode)


def level_info(cfg: OrcConfig) -> dict:
    L = cfg.nlevels
    w = np.zeros(L, np.int32); h = np.zeros(L, np.int32)
    s = np.zeros(L, np.float32); inv = np.zeros(L, np.float32)
    s2 = np.zeros(L, np.float32); is2 = np.zeros(L, np.float32)
    nf = np.zeros(L, np.int32); umax = np.zeros(16, np.int32)
    lib().orc_level_info(C.byref(cfg), _p(w), _p(h), _p(s), _p(inv), _p(s2), _p(is2), _p(nf), _p(umax))
    return dict(w=w, h=h, scale=s, inv_scale=inv, sigma2=s2, inv_sigma2=is2, nfeat=nf, umax=umax)


def extract(cfg: OrcConfig, img: np.ndarray):
    img = np.ascontiguousarray(img, np.uint8)
    cap = max(16 * cfg.nfeatures, 4096)
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = C.c_int(0)
    rc = lib().orc_extract(C.byref(cfg), _p(img), img.shape[1], img.shape[0],
                           C.c_size_t(img.strides[0]), _p(kps), cap, _p(desc), C.byref(n))
    assert rc == 0, rc
    return kps[:n.value].copy(), desc[:n.value].copy()


def pyramid_level(cfg: OrcConfig, img: np.ndarray, level: int) -> np.ndarray:
    info = level_info(cfg)
    out = np.zeros((info["h"][level], info["w"][level]), np.uint8)
    img = np.ascontiguousarray(img, np.uint8)
    lib().orc_pyramid_level(C.byref(cfg), _p(img), img.shape[1], img.shape[0],
                            C.c_size_t(img.strides[0]), level, _p(out))
    return out


def blur_level(cfg: OrcConfig, img: np.ndarray, level: int) -> np.ndarray:
    info = level_info(cfg)
    out = np.zeros((info["h"][level], info["w"][level]), np.uint8)
    img = np.ascontiguousarray(img, np.uint8)
    lib().orc_blur_level(C.byref(cfg), _p(img), img.shape[1], img.shape[0],
                         C.c_size_t(img.strides[0]), level, _p(out))
    return out


def fast_level(cfg: OrcConfig, img: np.ndarray, level: int) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    cap = 1 << 20
    kps = np.zeros(cap, KP_DTYPE)
    n = C.c_int(0)
    rc = lib().orc_fast_level(C.byref(cfg), _p(img), img.shape[1], img.shape[0],
                              C.c_size_t(img.strides[0]), level, _p(kps), cap, C.byref(n))
    assert rc == 0
    return kps[:n.value].copy()


def distribute(keys: np.ndarray, minX: int, maxX: int, minY: int, maxY: int, N: int) -> np.ndarray:
    keys = np.ascontiguousarray(keys, KP_DTYPE)
    cap = max(len(keys), N) + 8
    out = np.zeros(cap, KP_DTYPE)
    n = C.c_int(0)
    rc = lib().orc_distribute(_p(keys), len(keys), minX, maxX, minY, maxY, N, _p(out), cap, C.byref(n))
    assert rc == 0
    return out[:n.value].copy()


def tie_stats(cfg: OrcConfig, img: np.ndarray) -> dict:
    """Per-level tie-straddle exposure of the quadtree's creation-order tie rule
    (orb_oracle.h orc_extract_tie_stats): events, group nodes, kept keypoints."""
    img = np.ascontiguousarray(img, np.uint8)
    L = cfg.nlevels
    ev, nd, kp = (np.zeros(L, np.int32) for _ in range(3))
    lib().orc_extract_tie_stats(C.byref(cfg), _p(img), img.shape[1], img.shape[0], C.c_size_t(img.strides[0]),
                                _p(ev), _p(nd), _p(kp))
    return dict(events=ev, nodes=nd, kps=kp)


TIE_LATER_FIRST, TIE_POINTER, TIE_EARLIER_FIRST = 0, 1, 2


def extract_rule(cfg: OrcConfig, img: np.ndarray, tie_rule: int):
    """orc_extract with the quadtree's size ties broken by `tie_rule`
    (0 creation order later-first = the product's, 1 real heap address as the
    reference, 2 creation order earlier-first)."""
    img = np.ascontiguousarray(img, np.uint8)
    cap = max(16 * cfg.nfeatures, 4096)
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = C.c_int(0)
    rc = lib().orc_extract_rule(C.byref(cfg), tie_rule, _p(img), img.shape[1], img.shape[0],
                                C.c_size_t(img.strides[0]), _p(kps), cap, _p(desc), C.byref(n))
    assert rc == 0, rc
    return kps[:n.value].copy(), desc[:n.value].copy()


def tie_sequence(cfg: OrcConfig, frames: np.ndarray, rule_a: int, rule_b: int):
    """orc_tie_sequence: per (frame, level) whether rule_a and rule_b keep
    different keypoint lists, and how many positions only one of them kept."""
    frames = np.ascontiguousarray(frames, np.uint8)
    F, H, W = frames.shape
    L = cfg.nlevels
    differs = np.zeros((F, L), np.int32)
    kept = np.zeros((F, L), np.int32)
    lib().orc_tie_sequence(C.byref(cfg), _p(frames), F, W, H, C.c_size_t(W), C.c_size_t(H * W), rule_a, rule_b,
                           _p(differs), _p(kept))
    return differs.astype(bool), kept


def distribute_ties(keys: np.ndarray, minX: int, maxX: int, minY: int, maxY: int, N: int):
    keys = np.ascontiguousarray(keys, KP_DTYPE)
    ev, nd, kp = C.c_int(0), C.c_int(0), C.c_int(0)
    lib().orc_distribute_ties(_p(keys), len(keys), minX, maxX, minY, maxY, N, C.byref(ev), C.byref(nd), C.byref(kp))
    return ev.value, nd.value, kp.value


def pattern(pattern_mode: int = 0) -> np.ndarray:
    """The oracle's rBRIEF table, 1024 int8 entries in the reference's flat order."""
    out = np.zeros(1024, np.int8)
    lib().orc_pattern(pattern_mode, _p(out))
    return out


def descriptor_distance(a: np.ndarray, b: np.ndarray) -> int:
    a = np.ascontiguousarray(a, np.uint8); b = np.ascontiguousarray(b, np.uint8)
    return lib().orc_descriptor_distance(_p(a), _p(b))


def fast_atan2(y: float, x: float) -> float:
    return lib().orc_fast_atan2(y, x)


def hamming_top2(A: np.ndarray, B: np.ndarray):
    A = np.ascontiguousarray(A, np.uint8); B = np.ascontiguousarray(B, np.uint8)
    nA = len(A)
    bi = np.zeros(nA, np.int32); bd = np.zeros(nA, np.int32); sd = np.zeros(nA, np.int32)
    lib().orc_hamming_top2(_p(A), nA, _p(B), len(B), _p(bi), _p(bd), _p(sd))
    return bi, bd, sd


def search_for_initialization(kp1, desc1, kp2, desc2, bounds, prev_xy, window=100,
                              nnratio=0.9, check_ori=True):
    """Returns (matches12, nmatches, updated prev_xy). bounds = (minX, maxX, minY, maxY)."""
    kp1 = np.ascontiguousarray(kp1, KP_DTYPE); kp2 = np.ascontiguousarray(kp2, KP_DTYPE)
    desc1 = np.ascontiguousarray(desc1, np.uint8); desc2 = np.ascontiguousarray(desc2, np.uint8)
    prev = np.ascontiguousarray(prev_xy, np.float32).copy()
    m12 = np.zeros(len(kp1), np.int32)
    nm = C.c_int(0)
    lib().orc_search_for_initialization(
        _p(kp1), _p(desc1), len(kp1), _p(kp2), _p(desc2), len(kp2),
        C.c_float(bounds[0]), C.c_float(bounds[1]), C.c_float(bounds[2]), C.c_float(bounds[3]),
        _p(prev), window, C.c_float(nnratio), int(check_ori), _p(m12), C.byref(nm))
    return m12, nm.value, prev


def pyramid(cfg: OrcConfig, img: np.ndarray) -> list:
    """All levels of ComputePyramid as packed 2-D arrays (level 0 = the image)."""
    return [np.ascontiguousarray(img, np.uint8)] + [pyramid_level(cfg, img, l) for l in range(1, cfg.nlevels)]


def compute_stereo_matches(kpL, descL, kpR, descR, pyrL, pyrR, scale, inv_scale, mb, mbf):
    """Frame::ComputeStereoMatches. pyrL/pyrR: lists of per-level 2-D u8 arrays.
    Returns (mvuRight, mvDepth, kept)."""
    kpL = np.ascontiguousarray(kpL, KP_DTYPE); kpR = np.ascontiguousarray(kpR, KP_DTYPE)
    descL = np.ascontiguousarray(descL, np.uint8); descR = np.ascontiguousarray(descR, np.uint8)
    L = len(pyrL)
    pl = [np.ascontiguousarray(a, np.uint8) for a in pyrL]
    pr = [np.ascontiguousarray(a, np.uint8) for a in pyrR]
    ptrL = (C.c_void_p * L)(*[a.ctypes.data for a in pl])
    ptrR = (C.c_void_p * L)(*[a.ctypes.data for a in pr])
    sL = np.array([a.strides[0] for a in pl], np.uint64)
    sR = np.array([a.strides[0] for a in pr], np.uint64)
    lw = np.array([a.shape[1] for a in pl], np.int32)
    lh = np.array([a.shape[0] for a in pl], np.int32)
    sc = np.ascontiguousarray(scale, np.float32); isc = np.ascontiguousarray(inv_scale, np.float32)
    uR = np.zeros(len(kpL), np.float32); dep = np.zeros(len(kpL), np.float32)
    kept = lib().orc_compute_stereo_matches(_p(kpL), _p(descL), len(kpL), _p(kpR), _p(descR), len(kpR),
                                            ptrL, _p(sL), ptrR, _p(sR), _p(lw), _p(lh), L, _p(sc), _p(isc),
                                            C.c_float(mb), C.c_float(mbf), _p(uR), _p(dep))
    return uR, dep, kept


def search_by_bow(descA, angleA, mpA, fvA, descB, angleB, mpB, fvB, nnratio, check_ori,
                  kf_vs_kf):
    """fvX = (nodes u32, off i32, idx i32). Returns (out, nmatches)."""
    descA = np.ascontiguousarray(descA, np.uint8); descB = np.ascontiguousarray(descB, np.uint8)
    angleA = np.ascontiguousarray(angleA, np.float32); angleB = np.ascontiguousarray(angleB, np.float32)
    mpA = np.ascontiguousarray(mpA, np.uint8); mpB = np.ascontiguousarray(mpB, np.uint8)
    fa = [np.ascontiguousarray(x) for x in fvA]; fb = [np.ascontiguousarray(x) for x in fvB]
    nA, nB = len(descA), len(descB)
    out = np.zeros(nA if kf_vs_kf else nB, np.int32)
    nm = C.c_int(0)
    lib().orc_search_by_bow(_p(descA), _p(angleA), _p(mpA), nA, _p(fa[0]), _p(fa[1]), _p(fa[2]),
                            len(fa[0]), _p(descB), _p(angleB), _p(mpB), nB, _p(fb[0]), _p(fb[1]),
                            _p(fb[2]), len(fb[0]), C.c_float(nnratio), int(check_ori),
                            int(kf_vs_kf), _p(out), C.byref(nm))
    return out, nm.value


def sincosf(x):
    """Host libm sinf/cosf of a float32 array (returns sin, cos)."""
    x = np.ascontiguousarray(x, np.float32)
    s, c = np.empty_like(x), np.empty_like(x)
    lib().orc_sincosf(x.ctypes.data, len(x), s.ctypes.data, c.ctypes.data)
    return s, c


# ------------------------------------------------------------ DBoW2 vocabulary
def voc_load_text(path: str, cap: int = 2_000_000) -> dict:
    """TemplatedVocabulary::loadFromTextFile -> node arrays in file order."""
    k, L, sc, wt, n = (C.c_int(0) for _ in range(5))
    parent = np.zeros(cap, np.int32); leaf = np.zeros(cap, np.uint8)
    desc = np.zeros((cap, 32), np.uint8); weight = np.zeros(cap, np.float64)
    rc = lib().orc_voc_load_text(path.encode(), C.byref(k), C.byref(L), C.byref(sc), C.byref(wt), C.byref(n),
                                 cap, _p(parent), _p(leaf), _p(desc), _p(weight))
    if rc:
        raise ValueError(f"vocabulary load failed ({rc})")
    m = n.value
    return dict(k=k.value, L=L.value, scoring=sc.value, weighting=wt.value, parent=parent[:m].copy(),
                leaf=leaf[:m].copy(), desc=desc[:m].copy(), weight=weight[:m].copy())


def voc_transform(voc: dict, desc: np.ndarray, levelsup: int = 4) -> dict:
    """TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup).
    Returns per-feature word/nid/weight and the BowVector / FeatureVector (CSR)."""
    desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    n = len(desc)
    parent = np.ascontiguousarray(voc["parent"], np.int32)
    leaf = np.ascontiguousarray(voc["leaf"], np.uint8)
    nd = np.ascontiguousarray(voc["desc"], np.uint8)
    nw = np.ascontiguousarray(voc["weight"], np.float64)
    word = np.zeros(n, np.uint32); nid = np.zeros(n, np.uint32); w = np.zeros(n, np.float64)
    bw = np.zeros(max(n, 1), np.uint32); bv = np.zeros(max(n, 1), np.float64)
    fn = np.zeros(max(n, 1), np.uint32); fo = np.zeros(n + 1, np.int32); fi = np.zeros(max(n, 1), np.int32)
    nb, nf = C.c_int(0), C.c_int(0)
    lib().orc_voc_transform(voc["k"], voc["L"], voc["weighting"], voc["scoring"], len(parent), _p(parent),
                            _p(leaf), _p(nd), _p(nw), _p(desc), n, levelsup, _p(word), _p(nid), _p(w), _p(bw),
                            _p(bv), C.byref(nb), _p(fn), _p(fo), _p(fi), C.byref(nf))
    b, f = nb.value, nf.value
    return dict(word=word, nid=nid, weight=w, bow_words=bw[:b].copy(), bow_values=bv[:b].copy(),
                fv_nodes=fn[:f].copy(), fv_off=fo[:f + 1].copy(), fv_idx=fi[:fo[f]].copy())


# ------------------------------------------------------------ SearchByProjection
MP_DTYPE = np.dtype([("proj_x", "<f4"), ("proj_y", "<f4"), ("proj_xr", "<f4"), ("view_cos", "<f4"),
                     ("predicted_level", "<i4"), ("track_in_view", "u1"), ("obs_positive", "u1"),
                     ("pad", "u1", (2,))])


def search_by_projection(kps, desc, uright, bounds, scale, blocked, mps, mpdesc, th=1.0, nnratio=0.8):
    """ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th). Returns (out, nmatches):
    out[idx] = index of the map point the keypoint got in this call, -1 if none."""
    kps = np.ascontiguousarray(kps, KP_DTYPE); desc = np.ascontiguousarray(desc, np.uint8)
    ur = None if uright is None else np.ascontiguousarray(uright, np.float32)
    sc = np.ascontiguousarray(scale, np.float32); bl = np.ascontiguousarray(blocked, np.uint8)
    mps = np.ascontiguousarray(mps, MP_DTYPE); mpd = np.ascontiguousarray(mpdesc, np.uint8)
    out = np.zeros(max(len(kps), 1), np.int32)
    nm = C.c_int(0)
    lib().orc_search_by_projection(_p(kps), _p(desc), len(kps), None if ur is None else _p(ur),
                                   *[C.c_float(b) for b in bounds], _p(sc), _p(bl), _p(mps), _p(mpd), len(mps),
                                   C.c_float(th), C.c_float(nnratio), _p(out), C.byref(nm))
    return out[:len(kps)].copy(), nm.value


# ------------------------------------------------ SearchByProjection, pose overloads
MPW_DTYPE = np.dtype([("pos", "<f4", (3,)), ("normal", "<f4", (3,)), ("min_distance", "<f4"),
                      ("max_distance", "<f4"), ("angle", "<f4"), ("octave", "<i4"), ("valid", "u1"),
                      ("obs_positive", "u1"), ("pad", "u1", (6,))])
assert MPW_DTYPE.itemsize == 48


class OrcCamera(C.Structure):
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("mb", C.c_float), ("mbf", C.c_float), ("Tcw", C.c_float * 12)]


def camera(fx, fy, cx, cy, mb, mbf, Tcw) -> OrcCamera:
    T = np.asarray(Tcw, np.float32).reshape(-1)[:12]
    return OrcCamera(fx, fy, cx, cy, mb, mbf, (C.c_float * 12)(*T.tolist()))


def predict_scale(max_distance, dist, scale_factor=1.2, nlevels=8):
    lib().orc_predict_scale.argtypes = [C.c_float, C.c_float, C.c_float, C.c_int]
    return lib().orc_predict_scale(max_distance, dist, scale_factor, nlevels)


def predict_scale_ratios(ratios, scale_factor=1.2, nlevels=8):
    r = np.ascontiguousarray(ratios, np.float32)
    out = np.zeros(len(r), np.int32)
    f = lib().orc_predict_scale_ratios
    f.argtypes = [C.c_void_p, C.c_int, C.c_float, C.c_int, C.c_void_p]
    f(_p(r), len(r), scale_factor, nlevels, _p(out))
    return out


def _pose_common(kps, desc, mps, mpdesc):
    kps = np.ascontiguousarray(kps, KP_DTYPE); desc = np.ascontiguousarray(desc, np.uint8)
    mps = np.ascontiguousarray(mps, MPW_DTYPE); mpd = np.ascontiguousarray(mpdesc, np.uint8)
    return kps, desc, mps, mpd, np.zeros(max(len(kps), 1), np.int32), C.c_int(0)


def search_by_projection_last_frame(kps, desc, uright, bounds, scale, blocked, cam, Tlw, mps, mpdesc, th,
                                    mono, check_ori=True):
    """SearchByProjection(CurrentFrame, LastFrame, th, bMono). Returns (out, nmatches): out[i2] =
    last-frame index whose point the keypoint got, -1 untouched, -2 cleared by the rotation check."""
    kps, desc, mps, mpd, out, nm = _pose_common(kps, desc, mps, mpdesc)
    ur = None if uright is None else np.ascontiguousarray(uright, np.float32)
    sc = np.ascontiguousarray(scale, np.float32); bl = np.ascontiguousarray(blocked, np.uint8)
    T = np.ascontiguousarray(Tlw, np.float32).reshape(-1)
    f = lib().orc_search_by_projection_last_frame
    f.argtypes = ([C.c_void_p] * 2 + [C.c_int, C.c_void_p] + [C.c_float] * 4 + [C.c_void_p] * 6
                  + [C.c_int, C.c_float, C.c_int, C.c_int, C.c_void_p, C.c_void_p])
    f(_p(kps), _p(desc), len(kps), None if ur is None else _p(ur), *[C.c_float(b) for b in bounds], _p(sc),
      _p(bl), C.byref(cam), _p(T), _p(mps), _p(mpd), len(mps), th, int(mono), int(check_ori), _p(out),
      C.byref(nm))
    return out[:len(kps)].copy(), nm.value


def search_by_projection_keyframe(kps, desc, bounds, scale, scale_factor, has_mp, cam, mps, mpdesc, th, orb_dist,
                                  check_ori=True):
    """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (relocalization)."""
    kps, desc, mps, mpd, out, nm = _pose_common(kps, desc, mps, mpdesc)
    sc = np.ascontiguousarray(scale, np.float32); hm = np.ascontiguousarray(has_mp, np.uint8)
    f = lib().orc_search_by_projection_keyframe
    f.argtypes = ([C.c_void_p] * 2 + [C.c_int] + [C.c_float] * 4 + [C.c_void_p, C.c_int, C.c_float]
                  + [C.c_void_p] * 4 + [C.c_int, C.c_float, C.c_int, C.c_int, C.c_void_p, C.c_void_p])
    f(_p(kps), _p(desc), len(kps), *[C.c_float(b) for b in bounds], _p(sc), len(sc), scale_factor, _p(hm),
      C.byref(cam), _p(mps), _p(mpd), len(mps), th, int(orb_dist), int(check_ori), _p(out), C.byref(nm))
    return out[:len(kps)].copy(), nm.value


def search_by_projection_sim3(kps, desc, bounds, scale, scale_factor, cam, mps, mpdesc, th, matched=None):
    """SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (loop closing); cam.Tcw = Scw."""
    kps, desc, mps, mpd, out, nm = _pose_common(kps, desc, mps, mpdesc)
    sc = np.ascontiguousarray(scale, np.float32)
    mt = None if matched is None else np.ascontiguousarray(matched, np.int32)
    f = lib().orc_search_by_projection_sim3
    f.argtypes = ([C.c_void_p] * 2 + [C.c_int] + [C.c_float] * 4 + [C.c_void_p, C.c_int, C.c_float]
                  + [C.c_void_p] * 3 + [C.c_int, C.c_int] + [C.c_void_p] * 3)
    f(_p(kps), _p(desc), len(kps), *[C.c_float(b) for b in bounds], _p(sc), len(sc), scale_factor,
      C.byref(cam), _p(mps), _p(mpd), len(mps), int(th), None if mt is None else _p(mt), _p(out), C.byref(nm))
    return out[:len(kps)].copy(), nm.value


# ------------------------------------- Fuse, SearchBySim3, SearchForTriangulation
def fuse(kps, desc, uright, bounds, scale, inv_sigma2, scale_factor, cam, mps, mpdesc, th):
    """Fuse(pKF, vpMapPoints, th), match part: (out[i] = bestIdx or -1, nfused)."""
    kps, desc, mps, mpd, _, nm = _pose_common(kps, desc, mps, mpdesc)
    out = np.zeros(max(len(mps), 1), np.int32)
    ur = None if uright is None else np.ascontiguousarray(uright, np.float32)
    sc = np.ascontiguousarray(scale, np.float32); isg = np.ascontiguousarray(inv_sigma2, np.float32)
    f = lib().orc_fuse
    f.argtypes = ([C.c_void_p] * 2 + [C.c_int, C.c_void_p] + [C.c_float] * 4 + [C.c_void_p] * 2
                  + [C.c_int, C.c_float] + [C.c_void_p] * 3 + [C.c_int, C.c_float, C.c_void_p, C.c_void_p])
    f(_p(kps), _p(desc), len(kps), None if ur is None else _p(ur), *[C.c_float(b) for b in bounds], _p(sc),
      _p(isg), len(sc), scale_factor, C.byref(cam), _p(mps), _p(mpd), len(mps), th, _p(out), C.byref(nm))
    return out[:len(mps)].copy(), nm.value


def fuse_sim3(kps, desc, bounds, scale, scale_factor, cam, mps, mpdesc, th):
    """Fuse(pKF, Scw, vpPoints, th, vpReplacePoint), match part: (out[i] = bestIdx or -1, nfused)."""
    kps, desc, mps, mpd, _, nm = _pose_common(kps, desc, mps, mpdesc)
    out = np.zeros(max(len(mps), 1), np.int32)
    sc = np.ascontiguousarray(scale, np.float32)
    f = lib().orc_fuse_sim3
    f.argtypes = ([C.c_void_p] * 2 + [C.c_int] + [C.c_float] * 4 + [C.c_void_p, C.c_int, C.c_float]
                  + [C.c_void_p] * 3 + [C.c_int, C.c_float, C.c_void_p, C.c_void_p])
    f(_p(kps), _p(desc), len(kps), *[C.c_float(b) for b in bounds], _p(sc), len(sc), scale_factor, C.byref(cam),
      _p(mps), _p(mpd), len(mps), th, _p(out), C.byref(nm))
    return out[:len(mps)].copy(), nm.value


def search_by_sim3(kf1, kf2, cam1, s12, R12, t12, th, scale_factor=1.2):
    """SearchBySim3. kf1/kf2: dicts with kps, desc, bounds, scale, Tcw (3x4), mps, mpdesc (one record per
    keypoint). Returns (match1, nfound, vnMatch1, vnMatch2)."""
    k1 = np.ascontiguousarray(kf1["kps"], KP_DTYPE); k2 = np.ascontiguousarray(kf2["kps"], KP_DTYPE)
    d1 = np.ascontiguousarray(kf1["desc"], np.uint8); d2 = np.ascontiguousarray(kf2["desc"], np.uint8)
    b1 = np.asarray(kf1["bounds"], np.float32); b2 = np.asarray(kf2["bounds"], np.float32)
    s1 = np.ascontiguousarray(kf1["scale"], np.float32); s2 = np.ascontiguousarray(kf2["scale"], np.float32)
    T1 = np.ascontiguousarray(kf1["Tcw"], np.float32).reshape(-1); T2 = np.ascontiguousarray(kf2["Tcw"], np.float32).reshape(-1)
    m1 = np.ascontiguousarray(kf1["mps"], MPW_DTYPE); m2 = np.ascontiguousarray(kf2["mps"], MPW_DTYPE)
    q1 = np.ascontiguousarray(kf1["mpdesc"], np.uint8); q2 = np.ascontiguousarray(kf2["mpdesc"], np.uint8)
    R = np.ascontiguousarray(R12, np.float32).reshape(-1); t = np.ascontiguousarray(t12, np.float32).reshape(-1)
    match1 = np.zeros(max(len(k1), 1), np.int32); v1 = np.zeros(max(len(k1), 1), np.int32)
    v2 = np.zeros(max(len(k2), 1), np.int32); nf = C.c_int(0)
    f = lib().orc_search_by_sim3
    f.argtypes = ([C.c_void_p] * 2 + [C.c_int] + [C.c_void_p] * 4 + [C.c_int] + [C.c_void_p] * 2
                  + [C.c_int, C.c_float] + [C.c_void_p] * 3 + [C.c_float] + [C.c_void_p] * 6 + [C.c_float]
                  + [C.c_void_p] * 4)
    f(_p(k1), _p(d1), len(k1), _p(b1), _p(s1), _p(k2), _p(d2), len(k2), _p(b2), _p(s2), len(s1), scale_factor,
      C.byref(cam1), _p(T1), _p(T2), s12, _p(R), _p(t), _p(m1), _p(q1), _p(m2), _p(q2), th, _p(match1), _p(v1),
      _p(v2), C.byref(nf))
    return match1[:len(k1)].copy(), nf.value, v1[:len(k1)].copy(), v2[:len(k2)].copy()


def search_for_triangulation(kf1, kf2, cw1, T2w, cam2, sigma2, F12, only_stereo=False, check_ori=True):
    """SearchForTriangulation. kf: dicts with kps, desc, uright, has_mp and fv = (nodes, off, idx) CSR;
    kf2 also scale. Returns (matches12, nmatches)."""
    def arrs(kf):
        nodes, off, idx = kf["fv"]
        return (np.ascontiguousarray(kf["kps"], KP_DTYPE), np.ascontiguousarray(kf["desc"], np.uint8),
                np.ascontiguousarray(kf["uright"], np.float32), np.ascontiguousarray(kf["has_mp"], np.uint8),
                np.ascontiguousarray(nodes, np.uint32), np.ascontiguousarray(off, np.int32),
                np.ascontiguousarray(idx, np.int32) if len(idx) else np.zeros(1, np.int32))
    a1, a2 = arrs(kf1), arrs(kf2)
    out = np.zeros(max(len(a1[0]), 1), np.int32); nm = C.c_int(0)
    vec = lambda a: np.ascontiguousarray(a, np.float32).reshape(-1)
    cw, T, cm, sc2, sg2, F = vec(cw1), vec(T2w), vec(cam2), vec(kf2["scale"]), vec(sigma2), vec(F12)
    f = lib().orc_search_for_triangulation
    f.argtypes = ([C.c_void_p] * 4 + [C.c_int] + [C.c_void_p] * 3 + [C.c_int]) * 2 + [C.c_void_p] * 6 + \
        [C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    f(_p(a1[0]), _p(a1[1]), _p(a1[2]), _p(a1[3]), len(a1[0]), _p(a1[4]), _p(a1[5]), _p(a1[6]), len(a1[4]),
      _p(a2[0]), _p(a2[1]), _p(a2[2]), _p(a2[3]), len(a2[0]), _p(a2[4]), _p(a2[5]), _p(a2[6]), len(a2[4]),
      _p(cw), _p(T), _p(cm), _p(sc2), _p(sg2), _p(F), int(only_stereo), int(check_ori), _p(out), C.byref(nm))
    return out[:len(a1[0])].copy(), nm.value
