"""Second, independent restatement of the reference path in numpy / pure Python.

Used only by tests/test_oracle.py to cross-check the C++ oracle on small
inputs (it is far too slow for full frames). Each function follows the same
reference lines as the oracle, written from the reference text again rather
than from the oracle's code, so a slip in either shows up as a mismatch.
"""
from __future__ import annotations

import math

import numpy as np

f32 = np.float32


def cv_round(v) -> int:
    return int(np.rint(v))  # round half to even, like cvRound


# -------------------------------------------------------------- resize
def resize_linear_u8(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    """cv::resize INTER_LINEAR on u8 (OpenCV 3.x scalar fixed point)."""
    sh, sw = src.shape
    sx_scale, sy_scale = 1.0 / (dw / sw), 1.0 / (dh / sh)
    xofs = np.zeros(dw, np.int64)
    a = np.zeros((dw, 2), np.int64)
    xmax = dw
    for dx in range(dw):
        fx = f32((dx + 0.5) * sx_scale - 0.5)
        sx = int(math.floor(fx))
        fx = f32(fx - f32(sx))
        if sx < 0:
            fx, sx = f32(0), 0
        if sx + 1 >= sw:
            xmax = min(xmax, dx)
            if sx >= sw - 1:
                fx, sx = f32(0), sw - 1
        xofs[dx] = sx
        a[dx] = (cv_round(f32(f32(1) - fx) * f32(2048)), cv_round(fx * f32(2048)))
    out = np.zeros((dh, dw), np.uint8)
    S = src.astype(np.int64)
    cols = np.arange(dw)
    inside = cols < xmax
    nxt = np.minimum(xofs + 1, sw - 1)
    for dy in range(dh):
        fy = f32((dy + 0.5) * sy_scale - 0.5)
        sy = int(math.floor(fy))
        fy = f32(fy - f32(sy))
        b0, b1 = cv_round(f32(f32(1) - fy) * f32(2048)), cv_round(fy * f32(2048))
        rows = []
        for r in (min(max(sy, 0), sh - 1), min(max(sy + 1, 0), sh - 1)):
            R = S[r]
            rows.append(np.where(inside, R[xofs] * a[:, 0] + R[nxt] * a[:, 1], R[xofs] * 2048))
        out[dy] = np.clip((rows[0] * b0 + rows[1] * b1 + (1 << 21)) >> 22, 0, 255)
    return out


# -------------------------------------------------------------- blur
GAUSS7 = np.array([18, 34, 49, 55, 49, 34, 18], np.int64)


def gaussian_blur7(img: np.ndarray) -> np.ndarray:
    """GaussianBlur 7x7 sigma 2 BORDER_REFLECT_101, 8U fixed point."""
    p = np.pad(img.astype(np.int64), 3, mode="reflect")  # numpy 'reflect' == REFLECT_101
    H, W = img.shape
    row = sum(GAUSS7[i] * p[:, i:i + W] for i in range(7))
    col = sum(GAUSS7[i] * row[i:i + H, :] for i in range(7))
    return np.clip((col + (1 << 15)) >> 16, 0, 255).astype(np.uint8)


# -------------------------------------------------------------- FAST
RING = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
        (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def fast_score(img, x, y, t):
    """FAST-9 score of OpenCV (largest threshold still detecting, minus 1) or 0."""
    v = int(img[y, x])
    d = [v - int(img[y + dy, x + dx]) for dx, dy in RING]
    best = -1
    for s in range(16):
        arc = [d[(s + k) % 16] for k in range(9)]
        best = max(best, min(arc), -max(arc))
    # detected at t <=> some arc has all |d| > t in one direction
    return best - 1 if best - 1 >= t else 0


def fast_roi(img, x0, y0, cols, rows, t):
    """cv::FAST(ROI, t, nonmax=true): keypoints (x, y, score) in ROI coordinates."""
    sc = np.zeros((rows, cols), np.int64)
    for i in range(3, rows - 3):
        for j in range(3, cols - 3):
            sc[i, j] = fast_score(img, x0 + j, y0 + i, t)
    out = []
    for i in range(3, rows - 3):
        for j in range(3, cols - 3):
            s = sc[i, j]
            if s and all(s > sc[i + a, j + b] for a in (-1, 0, 1) for b in (-1, 0, 1) if a or b):
                out.append((j, i, s))
    return out


def fast_level(img, ini=20, mn=7, W=30.0):
    """FAST + per-cell grid of ComputeKeyPointsOctTree for one level."""
    minB = 16
    maxBX, maxBY = img.shape[1] - 16, img.shape[0] - 16
    width, height = f32(maxBX - minB), f32(maxBY - minB)
    nCols, nRows = int(width / f32(W)), int(height / f32(W))
    wCell, hCell = int(math.ceil(f32(width / f32(nCols)))), int(math.ceil(f32(height / f32(nRows))))
    keys = []
    for i in range(nRows):
        iniY = minB + i * hCell
        maxY = min(iniY + hCell + 6, maxBY)
        if iniY >= maxBY - 3:
            continue
        for j in range(nCols):
            iniX = minB + j * wCell
            maxX = min(iniX + wCell + 6, maxBX)
            if iniX >= maxBX - 6:
                continue
            k = fast_roi(img, iniX, iniY, maxX - iniX, maxY - iniY, ini)
            if not k:
                k = fast_roi(img, iniX, iniY, maxX - iniX, maxY - iniY, mn)
            keys += [(x + j * wCell, y + i * hCell, s) for x, y, s in k]
    return keys, (minB, maxBX, minB, maxBY)


# -------------------------------------------------------------- quadtree
class _Node:
    __slots__ = ("x0", "y0", "x1", "y1", "keys", "seq")

    def __init__(self, x0, y0, x1, y1, keys, seq):
        self.x0, self.y0, self.x1, self.y1, self.keys, self.seq = x0, y0, x1, y1, keys, seq


def _divide(n):
    hx = int(math.ceil(f32(n.x1 - n.x0) / f32(2)))
    hy = int(math.ceil(f32(n.y1 - n.y0) / f32(2)))
    mx, my = n.x0 + hx, n.y0 + hy
    boxes = [(n.x0, n.y0, mx, my), (mx, n.y0, n.x1, my), (n.x0, my, mx, n.y1), (mx, my, n.x1, n.y1)]
    parts = [[], [], [], []]
    for k in n.keys:
        parts[(0 if k[0] < mx else 1) + (0 if k[1] < my else 2)].append(k)
    return boxes, parts


def distribute(keys, minX, maxX, minY, maxY, N):
    """DistributeOctTree with a Python list as the std::list (front = index 0)."""
    nIni = int(round(float(f32(maxX - minX) / f32(maxY - minY))))
    hX = f32(f32(maxX - minX) / f32(nIni))
    seq = [0]

    def nxt():
        seq[0] += 1
        return seq[0]

    roots = [_Node(int(hX * f32(i)), 0, int(hX * f32(i + 1)), maxY - minY, [], nxt()) for i in range(nIni)]
    for k in keys:
        roots[int(f32(k[0]) / hX)].keys.append(k)
    lst = [n for n in roots if n.keys]
    expand = []
    phase2 = False
    while True:
        prev = len(lst)
        if not phase2:
            expand = []
            new_front, kept = [], []
            for pos, n in enumerate(lst):
                # list size right now: pushed children + surviving old nodes (incl. n)
                if len(new_front) + len(kept) + (len(lst) - pos) >= N:
                    kept += lst[pos:]
                    break
                if len(n.keys) == 1:
                    kept.append(n)
                    continue
                boxes, parts = _divide(n)
                for b, p in zip(boxes, parts):
                    if p:
                        c = _Node(*b, p, nxt())
                        new_front.insert(0, c)
                        if len(p) > 1:
                            expand.append(c)
            lst = new_front + kept
            if len(lst) >= N or len(lst) == prev:
                break
            if len(lst) + 3 * len(expand) > N:
                phase2 = True
        else:
            order = sorted(expand, key=lambda n: (len(n.keys), n.seq), reverse=True)
            expand = []
            for n in order:
                boxes, parts = _divide(n)
                for b, p in zip(boxes, parts):
                    if p:
                        c = _Node(*b, p, nxt())
                        lst.insert(0, c)
                        if len(p) > 1:
                            expand.append(c)
                lst.remove(n)
                if len(lst) >= N:
                    break
            if len(lst) >= N or len(lst) == prev:
                break
    out = []
    for n in lst:
        best = n.keys[0]
        for k in n.keys[1:]:
            if k[2] > best[2]:
                best = k
        out.append(best)
    return out


# -------------------------------------------------------------- matchers
def hamming(a, b) -> int:
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def three_maxima(hist):
    m = [0, 0, 0]
    ind = [-1, -1, -1]
    for i, s in enumerate(hist):
        if s > m[0]:
            m = [s, m[0], m[1]]
            ind = [i, ind[0], ind[1]]
        elif s > m[1]:
            m = [m[0], s, m[1]]
            ind = [ind[0], i, ind[1]]
        elif s > m[2]:
            m[2] = s
            ind[2] = i
    if m[1] < f32(0.1) * f32(m[0]):
        ind[1] = ind[2] = -1
    elif m[2] < f32(0.1) * f32(m[0]):
        ind[2] = -1
    return ind


def rot_bin(a1, a2):
    rot = f32(f32(a1) - f32(a2))
    if rot < 0:
        rot = f32(rot + f32(360))
    v = float(f32(rot * f32(f32(1) / f32(30))))
    b = int(math.floor(v + 0.5))  # round(): half away from zero (v >= 0)
    return 0 if b == 30 else b


def search_for_initialization(kp1, d1, kp2, d2, bounds, prev, r, ratio, check_ori):
    minX, maxX, minY, maxY = (f32(b) for b in bounds)
    invW, invH = f32(f32(64) / f32(maxX - minX)), f32(f32(48) / f32(maxY - minY))
    grid = [[[] for _ in range(48)] for _ in range(64)]
    for i, k in enumerate(kp2):
        gx = int(math.floor(float(f32(f32(k["x"]) - minX) * invW) + 0.5))
        gy = int(math.floor(float(f32(f32(k["y"]) - minY) * invH) + 0.5))
        if 0 <= gx < 64 and 0 <= gy < 48:
            grid[gx][gy].append(i)
    r = f32(r)
    m12 = [-1] * len(kp1)
    m21 = [-1] * len(kp2)
    md = [2 ** 31 - 1] * len(kp2)
    hist = [[] for _ in range(30)]
    nm = 0
    for i1, k1 in enumerate(kp1):
        if k1["octave"] > 0:
            continue
        x, y = f32(prev[i1][0]), f32(prev[i1][1])
        cx0 = max(0, int(math.floor(f32(f32(x - minX) - r) * invW)))
        cx1 = min(63, int(math.ceil(f32(f32(x - minX) + r) * invW)))
        cy0 = max(0, int(math.floor(f32(f32(y - minY) - r) * invH)))
        cy1 = min(47, int(math.ceil(f32(f32(y - minY) + r) * invH)))
        if cx0 >= 64 or cx1 < 0 or cy0 >= 48 or cy1 < 0:
            continue
        cand = [j for ix in range(cx0, cx1 + 1) for iy in range(cy0, cy1 + 1) for j in grid[ix][iy]
                if kp2[j]["octave"] == 0 and abs(f32(kp2[j]["x"]) - x) < r and abs(f32(kp2[j]["y"]) - y) < r]
        best, second, bi = 2 ** 31 - 1, 2 ** 31 - 1, -1
        for j in cand:
            d = hamming(d1[i1], d2[j])
            if md[j] <= d:
                continue
            if d < best:
                second, best, bi = best, d, j
            elif d < second:
                second = d
        if best <= 50 and f32(best) < f32(f32(second) * f32(ratio)):
            if m21[bi] >= 0:
                m12[m21[bi]] = -1
                nm -= 1
            m12[i1], m21[bi], md[bi] = bi, i1, best
            nm += 1
            if check_ori:
                hist[rot_bin(kp1[i1]["angle"], kp2[bi]["angle"])].append(i1)
    if check_ori:
        ind = three_maxima([len(h) for h in hist])
        for b in range(30):
            if b in ind:
                continue
            for i1 in hist[b]:
                if m12[i1] >= 0:
                    m12[i1] = -1
                    nm -= 1
    return np.array(m12, np.int32), nm


def search_by_bow(dA, angA, mpA, fvA, dB, angB, mpB, fvB, ratio, check_ori, kf_vs_kf):
    nodesA, offA, idxA = fvA
    nodesB, offB, idxB = fvB
    out = [-1] * (len(dA) if kf_vs_kf else len(dB))
    taken = [False] * len(dB)
    hist = [[] for _ in range(30)]
    nm = 0
    posB = {int(n): k for k, n in enumerate(nodesB)}
    for ka, n in enumerate(nodesA):
        kb = posB.get(int(n))
        if kb is None:
            continue
        for i1 in idxA[offA[ka]:offA[ka + 1]]:
            if not mpA[i1]:
                continue
            best, second, bi = 256, 256, -1
            for i2 in idxB[offB[kb]:offB[kb + 1]]:
                if taken[i2] or (kf_vs_kf and not mpB[i2]):
                    continue
                d = hamming(dA[i1], dB[i2])
                if d < best:
                    second, best, bi = best, d, i2
                elif d < second:
                    second = d
            ok = best < 50 if kf_vs_kf else best <= 50
            if ok and f32(best) < f32(f32(ratio) * f32(second)):
                taken[bi] = True
                if kf_vs_kf:
                    out[i1] = bi
                else:
                    out[bi] = i1
                nm += 1
                if check_ori:
                    hist[rot_bin(angA[i1], angB[bi])].append(i1 if kf_vs_kf else bi)
    if check_ori:
        ind = three_maxima([len(h) for h in hist])
        for b in range(30):
            if b in ind:
                continue
            for i in hist[b]:
                out[i] = -1
                nm -= 1
    return np.array(out, np.int32), nm


# -------------------------------------------------------------- stereo
def _c_round(v) -> float:
    """std::round on a float: half away from zero."""
    v = float(v)
    return math.copysign(math.floor(abs(v) + 0.5), v)


def compute_stereo_matches(kpL, dL, kpR, dR, pyrL, pyrR, scale, inv_scale, mb, mbf):
    """Frame::ComputeStereoMatches (src/Frame.cc:465-639). pyrL/pyrR: per-level 2-D u8.
    Windows reaching off the level (an OpenCV range assertion there) give no match."""
    nL = len(kpL)
    uR_out = np.full(nL, -1.0, np.float32)
    dep_out = np.full(nL, -1.0, np.float32)
    nrows = pyrL[0].shape[0]
    rows = [[] for _ in range(nrows)]
    for iR in range(len(kpR)):
        y = f32(kpR["y"][iR])
        r = f32(f32(2) * f32(scale[int(kpR["octave"][iR])]))
        for yi in range(int(math.floor(f32(y - r))), int(math.ceil(f32(y + r))) + 1):
            if 0 <= yi < nrows:
                rows[yi].append(iR)
    mb, mbf = f32(mb), f32(mbf)
    maxD = f32(mbf / mb)
    acc = []
    for iL in range(nL):
        lev = int(kpL["octave"][iL])
        uL, vL = f32(kpL["x"][iL]), f32(kpL["y"][iL])
        if not (0 <= vL < nrows):
            continue
        cands = rows[int(vL)]
        minU, maxU = f32(uL - maxD), uL
        if not cands or maxU < 0:
            continue
        best, bi = 100, 0
        for iR in cands:
            o = int(kpR["octave"][iR])
            if o < lev - 1 or o > lev + 1:
                continue
            u = f32(kpR["x"][iR])
            if minU <= u <= maxU:
                d = hamming(dL[iL], dR[iR])
                if d < best:
                    best, bi = d, iR
        if best >= 75:
            continue
        sf = f32(inv_scale[lev])
        su = _c_round(f32(uL * sf))
        sv = _c_round(f32(vL * sf))
        sr = _c_round(f32(f32(kpR["x"][bi]) * sf))
        A, B = pyrL[lev].astype(np.int64), pyrR[lev].astype(np.int64)
        h, w = A.shape
        ul, vl, ur = int(su), int(sv), int(sr)
        if ur < 10 or ul < 5 or ul + 5 >= w or vl < 5 or vl + 5 >= h:
            continue
        if sr < 0 or sr + 11 >= w:  # iniu / endu
            continue
        IL = A[vl - 5:vl + 6, ul - 5:ul + 6] - A[vl, ul]
        dists = []
        for inc in range(-5, 6):
            IR = B[vl - 5:vl + 6, ur + inc - 5:ur + inc + 6] - B[vl, ur + inc]
            dists.append(int(np.abs(IL - IR).sum()))
        binc = int(np.argmin(dists)) - 5  # first minimum
        bdist = min(dists)
        if binc in (-5, 5):
            continue
        d1, d2, d3 = (f32(dists[binc + 5 + k]) for k in (-1, 0, 1))
        with np.errstate(divide="ignore", invalid="ignore"):
            delta = f32(f32(d1 - d3) / f32(f32(2) * f32(f32(d1 + d3) - f32(f32(2) * d2))))
        if delta < -1 or delta > 1:
            continue
        buR = f32(f32(scale[lev]) * f32(f32(f32(sr) + f32(binc)) + delta))
        disp = f32(uL - buR)
        if disp >= 0 and disp < maxD:
            if disp <= 0:
                disp = f32(0.01)
                buR = f32(float(uL) - 0.01)
            dep_out[iL] = f32(mbf / disp)
            uR_out[iL] = buR
            acc.append((bdist, iL))
    if not acc:
        return uR_out, dep_out, 0
    acc.sort()
    th = f32(f32(f32(1.5) * f32(1.4)) * f32(acc[len(acc) // 2][0]))
    kept = len(acc)
    for d, i in reversed(acc):
        if f32(d) < th:
            break
        uR_out[i] = dep_out[i] = -1
        kept -= 1
    return uR_out, dep_out, kept


# -------------------------------------------------------------- DBoW2 transform
def voc_transform(voc, desc, levelsup):
    """TemplatedVocabulary::transform(features, v, fv, levelsup)
    (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1127-1256, BowVector.cpp,
    FeatureVector.cpp). Returns (words, nids, weights, bow dict, fv dict)."""
    n_nodes = len(voc["parent"])
    children = [[] for _ in range(n_nodes)]
    word_id = [0] * n_nodes
    nw = 0
    for i in range(1, n_nodes):
        children[int(voc["parent"][i])].append(i)
        if voc["leaf"][i]:
            word_id[i] = nw
            nw += 1
    nd = voc["desc"]
    words, nids, ws = [], [], []
    bow, fv = {}, {}
    if nw == 0:
        return words, nids, ws, bow, fv
    nid_level = voc["L"] - levelsup
    tf = voc["weighting"] in (0, 1)
    for i, f in enumerate(np.asarray(desc, np.uint8).reshape(-1, 32)):
        node, level, nid = 0, 0, 0
        while True:
            level += 1
            ch = children[node]
            dists = [hamming(f, nd[c]) for c in ch]
            node = ch[int(np.argmin(dists))]  # first minimum
            if level == nid_level:
                nid = node
            if not children[node]:
                break
        if nid_level > level:
            nid = node
        w = float(voc["weight"][node])
        words.append(word_id[node]); nids.append(nid); ws.append(w)
        if w > 0:
            if tf:
                bow[word_id[node]] = bow.get(word_id[node], 0.0) + w
            else:
                bow.setdefault(word_id[node], w)
            fv.setdefault(nid, []).append(i)
    must = voc["scoring"] != 5
    if tf and bow and not must:
        nb = float(len(bow))
        bow = {k: v / nb for k, v in bow.items()}
    if must:
        keys = sorted(bow)
        if voc["scoring"] == 1:
            norm = 0.0
            for k in keys:
                norm += bow[k] * bow[k]
            norm = math.sqrt(norm)
        else:
            norm = 0.0
            for k in keys:
                norm += abs(bow[k])
        if norm > 0.0:
            bow = {k: bow[k] / norm for k in keys}
    return words, nids, ws, bow, fv


# -------------------------------------------------------------- SearchByProjection
def features_in_area(kps, cells, bounds, x, y, r, minLevel, maxLevel):
    """Frame::GetFeaturesInArea (src/Frame.cc:326-379) over a prebuilt 64 x 48 grid."""
    minX, maxX, minY, maxY = (f32(b) for b in bounds)
    invW = f32(f32(64) / f32(maxX - minX))
    invH = f32(f32(48) / f32(maxY - minY))
    x, y, r = f32(x), f32(y), f32(r)
    cx0 = max(0, int(math.floor(f32(f32(f32(x - minX) - r) * invW))))
    if cx0 >= 64:
        return []
    cx1 = min(63, int(math.ceil(f32(f32(f32(x - minX) + r) * invW))))
    if cx1 < 0:
        return []
    cy0 = max(0, int(math.floor(f32(f32(f32(y - minY) - r) * invH))))
    if cy0 >= 48:
        return []
    cy1 = min(47, int(math.ceil(f32(f32(f32(y - minY) + r) * invH))))
    if cy1 < 0:
        return []
    check = minLevel > 0 or maxLevel >= 0
    out = []
    for ix in range(cx0, cx1 + 1):
        for iy in range(cy0, cy1 + 1):
            for j in cells.get((ix, iy), []):
                o = int(kps["octave"][j])
                if check and (o < minLevel or (maxLevel >= 0 and o > maxLevel)):
                    continue
                if abs(f32(f32(kps["x"][j]) - x)) < r and abs(f32(f32(kps["y"][j]) - y)) < r:
                    out.append(j)
    return out


def grid_cells(kps, bounds):
    """Frame::AssignFeaturesToGrid / PosInGrid (src/Frame.cc:228-243, 381-391)."""
    minX, maxX, minY, maxY = (f32(b) for b in bounds)
    invW = f32(f32(64) / f32(maxX - minX))
    invH = f32(f32(48) / f32(maxY - minY))
    cells = {}
    for i in range(len(kps)):
        px = _c_round(f32(f32(f32(kps["x"][i]) - minX) * invW))
        py = _c_round(f32(f32(f32(kps["y"][i]) - minY) * invH))
        if 0 <= px < 64 and 0 <= py < 48:
            cells.setdefault((int(px), int(py)), []).append(i)
    return cells


def search_by_projection(kps, desc, uright, bounds, scale, blocked, mps, mpdesc, th, ratio, independent=False):
    """ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th) (src/ORBmatcher.cc:45-118).
    independent=True drops the blocking by earlier points (a test of the test data only)."""
    cells = grid_cells(kps, bounds)
    blk = [bool(b) for b in blocked]
    out = [-1] * len(kps)
    nm = 0
    th = f32(th)
    for j in range(len(mps)):
        mp = mps[j]
        if not mp["track_in_view"]:
            continue
        lvl = int(mp["predicted_level"])
        r = f32(2.5) if float(f32(mp["view_cos"])) > 0.998 else f32(4.0)
        if float(th) != 1.0:
            r = f32(r * th)
        rad = f32(r * f32(scale[lvl]))
        idxs = features_in_area(kps, cells, bounds, mp["proj_x"], mp["proj_y"], rad, lvl - 1, lvl)
        best, bl, best2, bl2, bi = 256, -1, 256, -1, -1
        for i in idxs:
            if blk[i]:
                continue
            if uright is not None and uright[i] > 0:
                if abs(f32(f32(mp["proj_xr"]) - f32(uright[i]))) > rad:
                    continue
            d = hamming(mpdesc[j], desc[i])
            if d < best:
                best2, best, bl2, bl, bi = best, d, bl, int(kps["octave"][i]), i
            elif d < best2:
                bl2, best2 = int(kps["octave"][i]), d
        if best <= 100:
            if bl == bl2 and f32(best) > f32(f32(ratio) * f32(best2)):
                continue
            out[bi] = j
            if not independent:
                blk[bi] = bool(mp["obs_positive"])
            nm += 1
    return np.array(out, np.int32), nm


# ------------------------------------------- SearchByProjection, pose overloads
import ctypes as _C  # noqa: E402

_libm = _C.CDLL("libm.so.6")
_libm.logf.restype = _C.c_float
_libm.logf.argtypes = [_C.c_float]


def _logf(x):
    return f32(_libm.logf(float(f32(x))))


def _mat_rx_t(T, x):
    """R*x + t: OpenCV gemm small-matrix path (float dot, then double add of t)."""
    T = np.asarray(T, np.float32).reshape(3, 4)
    out = []
    for r in range(3):
        t = f32(f32(f32(T[r, 0] * f32(x[0])) + f32(T[r, 1] * f32(x[1]))) + f32(T[r, 2] * f32(x[2])))
        out.append(f32(float(t) + float(T[r, 3])))
    return out


def _mat_neg_rt_t(T):
    """-R.t()*t: general gemm path with double accumulation."""
    T = np.asarray(T, np.float32).reshape(3, 4)
    out = []
    for r in range(3):
        s = 0.0
        for k in range(3):
            s += float(T[k, r]) * float(T[k, 3])
        out.append(f32(-s))
    return out


def _norm3(v):
    s = 0.0
    for e in v:
        s += float(e) * float(e)
    return math.sqrt(s)


def _dot3(a, b):
    s = 0.0
    for x, y in zip(a, b):
        s += float(x) * float(y)
    return s


def predict_scale(maxd, dist, sf, L):
    """MapPoint::PredictScale (src/MapPoint.cc:407-422), float log."""
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio = f32(f32(maxd) / f32(dist))
        q = f32(_logf(ratio) / _logf(sf))
    if not np.isfinite(q):
        return 0  # x86 float->int of a non-finite value: INT_MIN, clamped to 0
    n = int(math.ceil(float(q)))
    return 0 if n < 0 else min(n, L - 1)


def _rot_filter(hist, out, nm):
    ind = three_maxima([len(h) for h in hist])
    for b in range(30):
        if b not in ind:
            for i2 in hist[b]:
                out[i2] = -2
                nm -= 1
    return nm


def _cam(cam):
    return (f32(cam.fx), f32(cam.fy), f32(cam.cx), f32(cam.cy), f32(cam.mb), f32(cam.mbf),
            np.array(list(cam.Tcw), np.float32))


def search_by_projection_last_frame(kps, desc, uright, bounds, scale, blocked, cam, Tlw, mps, mpdesc, th, mono,
                                    check_ori=True):
    """SearchByProjection(CurrentFrame, LastFrame, th, bMono) (src/ORBmatcher.cc:1328-1470)."""
    fx, fy, cx, cy, mb, mbf, T = _cam(cam)
    cells = grid_cells(kps, bounds)
    minX, maxX, minY, maxY = (f32(b) for b in bounds)
    twc = _mat_neg_rt_t(T)
    tlc = _mat_rx_t(np.asarray(Tlw, np.float32), twc)
    fwd = tlc[2] > mb and not mono
    bwd = -tlc[2] > mb and not mono
    blk = [bool(b) for b in blocked]
    out = [-1] * len(kps)
    hist = [[] for _ in range(30)]
    nm = 0
    th = f32(th)
    for i in range(len(mps)):
        mp = mps[i]
        if not mp["valid"]:
            continue
        xc, yc, zc = _mat_rx_t(T, mp["pos"])
        invzc = f32(1.0 / float(zc)) if zc != 0 else f32(math.copysign(math.inf, float(zc)))
        if invzc < 0:
            continue
        u = f32(f32(f32(fx * xc) * invzc) + cx)
        v = f32(f32(f32(fy * yc) * invzc) + cy)
        if u < minX or u > maxX or v < minY or v > maxY:
            continue
        lo = int(mp["octave"])
        rad = f32(th * f32(scale[lo]))
        if fwd:
            idxs = features_in_area(kps, cells, bounds, u, v, rad, lo, -1)
        elif bwd:
            idxs = features_in_area(kps, cells, bounds, u, v, rad, 0, lo)
        else:
            idxs = features_in_area(kps, cells, bounds, u, v, rad, lo - 1, lo + 1)
        best, bi = 256, -1
        for i2 in idxs:
            if blk[i2]:
                continue
            if uright is not None and uright[i2] > 0:
                ur = f32(u - f32(mbf * invzc))
                if abs(f32(ur - f32(uright[i2]))) > rad:
                    continue
            d = hamming(mpdesc[i], desc[i2])
            if d < best:
                best, bi = d, i2
        if best <= 100:
            out[bi] = i
            blk[bi] = bool(mp["obs_positive"])
            nm += 1
            if check_ori:
                hist[rot_bin(mp["angle"], kps["angle"][bi])].append(bi)
    if check_ori:
        nm = _rot_filter(hist, out, nm)
    return np.array(out, np.int32), nm


def search_by_projection_keyframe(kps, desc, bounds, scale, sf, has_mp, cam, mps, mpdesc, th, orb_dist,
                                  check_ori=True):
    """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (src/ORBmatcher.cc:1472-1599)."""
    fx, fy, cx, cy, mb, mbf, T = _cam(cam)
    cells = grid_cells(kps, bounds)
    minX, maxX, minY, maxY = (f32(b) for b in bounds)
    Ow = _mat_neg_rt_t(T)
    taken = [bool(b) for b in has_mp]
    out = [-1] * len(kps)
    hist = [[] for _ in range(30)]
    nm = 0
    th = f32(th)
    L = len(scale)
    for i in range(len(mps)):
        mp = mps[i]
        if not mp["valid"]:
            continue
        xc, yc, zc = _mat_rx_t(T, mp["pos"])
        invzc = f32(1.0 / float(zc)) if zc != 0 else f32(math.copysign(math.inf, float(zc)))
        u = f32(f32(f32(fx * xc) * invzc) + cx)
        v = f32(f32(f32(fy * yc) * invzc) + cy)
        if u < minX or u > maxX or v < minY or v > maxY:
            continue
        PO = [f32(f32(mp["pos"][k]) - Ow[k]) for k in range(3)]
        d3 = f32(_norm3(PO))
        if d3 < f32(f32(0.8) * f32(mp["min_distance"])) or d3 > f32(f32(1.2) * f32(mp["max_distance"])):
            continue
        lvl = predict_scale(mp["max_distance"], d3, sf, L)
        rad = f32(th * f32(scale[lvl]))
        best, bi = 256, -1
        for i2 in features_in_area(kps, cells, bounds, u, v, rad, lvl - 1, lvl + 1):
            if taken[i2]:
                continue
            d = hamming(mpdesc[i], desc[i2])
            if d < best:
                best, bi = d, i2
        if best <= orb_dist:
            out[bi] = i
            taken[bi] = True
            nm += 1
            if check_ori:
                hist[rot_bin(mp["angle"], kps["angle"][bi])].append(bi)
    if check_ori:
        nm = _rot_filter(hist, out, nm)
    return np.array(out, np.int32), nm


def search_by_projection_sim3(kps, desc, bounds, scale, sf, cam, mps, mpdesc, th, matched=None):
    """SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (src/ORBmatcher.cc:290-403)."""
    fx, fy, cx, cy, mb, mbf, S = _cam(cam)
    cells = grid_cells(kps, bounds)
    minX, maxX, minY, maxY = (f32(b) for b in bounds)
    scw = f32(math.sqrt(_dot3(S[0:3], S[0:3])))
    a = f32(1.0 / float(scw))
    T = np.array([f32(f32(s * a) + f32(0)) for s in S], np.float32)
    Ow = _mat_neg_rt_t(T)
    taken = [False] * len(kps) if matched is None else [int(m) >= 0 for m in matched]
    out = [-1] * len(kps)
    nm = 0
    L = len(scale)
    for i in range(len(mps)):
        mp = mps[i]
        if not mp["valid"]:
            continue
        X, Y, Z = _mat_rx_t(T, mp["pos"])
        if Z < 0.0:
            continue
        invz = f32(f32(1) / Z)
        u = f32(f32(fx * f32(X * invz)) + cx)
        v = f32(f32(fy * f32(Y * invz)) + cy)
        if not (u >= minX and u < maxX and v >= minY and v < maxY):
            continue
        PO = [f32(f32(mp["pos"][k]) - Ow[k]) for k in range(3)]
        dist = f32(_norm3(PO))
        if dist < f32(f32(0.8) * f32(mp["min_distance"])) or dist > f32(f32(1.2) * f32(mp["max_distance"])):
            continue
        if _dot3(PO, mp["normal"]) < 0.5 * float(dist):
            continue
        lvl = predict_scale(mp["max_distance"], dist, sf, L)
        rad = f32(f32(th) * f32(scale[lvl]))
        best, bi = 256, -1
        for idx in features_in_area(kps, cells, bounds, u, v, rad, -1, -1):
            if taken[idx]:
                continue
            o = int(kps["octave"][idx])
            if o < lvl - 1 or o > lvl:
                continue
            d = hamming(mpdesc[i], desc[idx])
            if d < best:
                best, bi = d, idx
        if best <= 50:
            out[bi] = i
            taken[bi] = True
            nm += 1
    return np.array(out, np.int32), nm


# ------------------------------------ Fuse, SearchBySim3, SearchForTriangulation
def _in_image(u, v, bounds):
    minX, maxX, minY, maxY = (f32(b) for b in bounds)
    return u >= minX and u < maxX and v >= minY and v < maxY


def _sim3_T(S):
    S = np.asarray(S, np.float32).reshape(-1)
    scw = f32(math.sqrt(_dot3(S[0:3], S[0:3])))
    a = f32(1.0 / float(scw))
    return np.array([f32(f32(s * a) + f32(0)) for s in S], np.float32)


def _dist_ok(mp, dist):
    return not (dist < f32(f32(0.8) * f32(mp["min_distance"])) or dist > f32(f32(1.2) * f32(mp["max_distance"])))


def _kf_best(kps, desc, cells, bounds, u, v, rad, lvl, dmp, init, extra=None):
    best, bi = init, -1
    for idx in features_in_area(kps, cells, bounds, u, v, rad, -1, -1):
        o = int(kps["octave"][idx])
        if o < lvl - 1 or o > lvl:
            continue
        if extra is not None and not extra(idx):
            continue
        d = hamming(dmp, desc[idx])
        if d < best:
            best, bi = d, idx
    return best, bi


def fuse(kps, desc, uright, bounds, scale, inv_sigma2, sf, cam, mps, mpdesc, th):
    """Fuse(pKF, vpMapPoints, th) (src/ORBmatcher.cc:825-930), match part."""
    fx, fy, cx, cy, mb, bf, T = _cam(cam)
    cells = grid_cells(kps, bounds)
    Ow = _mat_neg_rt_t(T)
    L = len(scale)
    out = [-1] * len(mps)
    nf = 0
    for i in range(len(mps)):
        mp = mps[i]
        if not mp["valid"]:
            continue
        X, Y, Z = _mat_rx_t(T, mp["pos"])
        if Z < f32(0):
            continue
        invz = f32(f32(1) / Z)
        u = f32(f32(fx * f32(X * invz)) + cx)
        v = f32(f32(fy * f32(Y * invz)) + cy)
        if not _in_image(u, v, bounds):
            continue
        ur = f32(u - f32(bf * invz))
        PO = [f32(f32(mp["pos"][k]) - Ow[k]) for k in range(3)]
        dist = f32(_norm3(PO))
        if not _dist_ok(mp, dist) or _dot3(PO, mp["normal"]) < 0.5 * float(dist):
            continue
        lvl = predict_scale(mp["max_distance"], dist, sf, L)
        rad = f32(f32(th) * f32(scale[lvl]))

        def reproj(idx):
            o = int(kps["octave"][idx])
            ex = f32(u - f32(kps["x"][idx]))
            ey = f32(v - f32(kps["y"][idx]))
            if uright is not None and uright[idx] >= 0:
                er = f32(ur - f32(uright[idx]))
                e2 = f32(f32(f32(ex * ex) + f32(ey * ey)) + f32(er * er))
                return not float(f32(e2 * f32(inv_sigma2[o]))) > 7.8
            e2 = f32(f32(ex * ex) + f32(ey * ey))
            return not float(f32(e2 * f32(inv_sigma2[o]))) > 5.99
        best, bi = _kf_best(kps, desc, cells, bounds, u, v, rad, lvl, mpdesc[i], 256, reproj)
        if best <= 50:
            out[i] = bi
            nf += 1
    return np.array(out, np.int32), nf


def fuse_sim3(kps, desc, bounds, scale, sf, cam, mps, mpdesc, th):
    """Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (src/ORBmatcher.cc:977-1081), match part."""
    fx, fy, cx, cy, mb, mbf, S = _cam(cam)
    T = _sim3_T(S)
    cells = grid_cells(kps, bounds)
    Ow = _mat_neg_rt_t(T)
    L = len(scale)
    out = [-1] * len(mps)
    nf = 0
    for i in range(len(mps)):
        mp = mps[i]
        if not mp["valid"]:
            continue
        X, Y, Z = _mat_rx_t(T, mp["pos"])
        if Z < f32(0):
            continue
        invz = f32(1.0 / float(Z))
        u = f32(f32(fx * f32(X * invz)) + cx)
        v = f32(f32(fy * f32(Y * invz)) + cy)
        if not _in_image(u, v, bounds):
            continue
        PO = [f32(f32(mp["pos"][k]) - Ow[k]) for k in range(3)]
        dist = f32(_norm3(PO))
        if not _dist_ok(mp, dist) or _dot3(PO, mp["normal"]) < 0.5 * float(dist):
            continue
        lvl = predict_scale(mp["max_distance"], dist, sf, L)
        rad = f32(f32(th) * f32(scale[lvl]))
        best, bi = _kf_best(kps, desc, cells, bounds, u, v, rad, lvl, mpdesc[i], 1 << 31)
        if best <= 50:
            out[i] = bi
            nf += 1
    return np.array(out, np.int32), nf


def search_by_sim3(kf1, kf2, cam1, s12, R12, t12, th, sf=1.2):
    """SearchBySim3 (src/ORBmatcher.cc:1102-1326)."""
    fx, fy, cx, cy = f32(cam1.fx), f32(cam1.fy), f32(cam1.cx), f32(cam1.cy)
    R = np.asarray(R12, np.float32).reshape(3, 3)
    t = np.asarray(t12, np.float32).reshape(3)
    a12, a21 = f32(s12), f32(1.0 / float(f32(s12)))
    S12 = np.zeros((3, 4), np.float32)
    S21 = np.zeros((3, 4), np.float32)
    for r in range(3):
        for c in range(3):
            S12[r, c] = f32(f32(R[r, c] * a12) + f32(0))
            S21[r, c] = f32(f32(R[c, r] * a21) + f32(0))
    for r in range(3):
        S12[r, 3] = t[r]
        d = f32(f32(f32(S21[r, 0] * t[0]) + f32(S21[r, 1] * t[1])) + f32(S21[r, 2] * t[2]))
        S21[r, 3] = f32(-float(d))

    def direction(A, B, S):
        cells = grid_cells(B["kps"], B["bounds"])
        L = len(B["scale"])
        vm = [-1] * len(A["kps"])
        for i in range(len(A["kps"])):
            mp = A["mps"][i]
            if not mp["valid"]:
                continue
            p1 = _mat_rx_t(np.asarray(A["Tcw"], np.float32), mp["pos"])
            p2 = _mat_rx_t(S, p1)
            if p2[2] < 0.0:
                continue
            invz = f32(1.0 / float(p2[2]))
            u = f32(f32(fx * f32(p2[0] * invz)) + cx)
            v = f32(f32(fy * f32(p2[1] * invz)) + cy)
            if not _in_image(u, v, B["bounds"]):
                continue
            dist = f32(_norm3(p2))
            if not _dist_ok(mp, dist):
                continue
            lvl = predict_scale(mp["max_distance"], dist, sf, L)
            rad = f32(f32(th) * f32(B["scale"][lvl]))
            best, bi = _kf_best(B["kps"], B["desc"], cells, B["bounds"], u, v, rad, lvl, A["mpdesc"][i], 1 << 31)
            if best <= 100:
                vm[i] = bi
        return vm
    v1 = direction(kf1, kf2, S21)
    v2 = direction(kf2, kf1, S12)
    m1 = [-1] * len(v1)
    nf = 0
    for i1, i2 in enumerate(v1):
        if i2 >= 0 and v2[i2] == i1:
            m1[i1] = i2
            nf += 1
    return np.array(m1, np.int32), nf


def search_for_triangulation(kf1, kf2, cw1, T2w, cam2, sigma2, F12, only_stereo=False, check_ori=True):
    """SearchForTriangulation (src/ORBmatcher.cc:657-823) + CheckDistEpipolarLine (:140-157)."""
    C2 = _mat_rx_t(np.asarray(T2w, np.float32), np.asarray(cw1, np.float32))
    invz = f32(f32(1) / C2[2])
    cam2 = np.asarray(cam2, np.float32)
    ex = f32(f32(f32(cam2[0] * C2[0]) * invz) + cam2[2])
    ey = f32(f32(f32(cam2[1] * C2[1]) * invz) + cam2[3])
    F = np.asarray(F12, np.float32).reshape(3, 3)
    k1, k2 = kf1["kps"], kf2["kps"]

    def epi(i1, i2):
        x1, y1 = f32(k1["x"][i1]), f32(k1["y"][i1])
        a = f32(f32(f32(x1 * F[0, 0]) + f32(y1 * F[1, 0])) + F[2, 0])
        b = f32(f32(f32(x1 * F[0, 1]) + f32(y1 * F[1, 1])) + F[2, 1])
        c = f32(f32(f32(x1 * F[0, 2]) + f32(y1 * F[1, 2])) + F[2, 2])
        num = f32(f32(f32(a * f32(k2["x"][i2])) + f32(b * f32(k2["y"][i2]))) + c)
        den = f32(f32(a * a) + f32(b * b))
        if den == 0:
            return False
        dsqr = f32(f32(num * num) / den)
        return float(dsqr) < 3.84 * float(f32(sigma2[int(k2["octave"][i2])]))
    n1, (nd1, of1, ix1), (nd2, of2, ix2) = len(k1), kf1["fv"], kf2["fv"]
    node2 = {int(n): j for j, n in enumerate(nd2)}
    m12 = [-1] * n1
    hist = [[] for _ in range(30)]
    nm = 0
    for a, node in enumerate(nd1):
        if int(node) not in node2:
            continue
        b = node2[int(node)]
        for i1 in ix1[of1[a]:of1[a + 1]]:
            if kf1["has_mp"][i1]:
                continue
            st1 = kf1["uright"][i1] >= 0
            if only_stereo and not st1:
                continue
            best, bi = 50, -1
            for i2 in ix2[of2[b]:of2[b + 1]]:
                if kf2["has_mp"][i2]:
                    continue
                st2 = kf2["uright"][i2] >= 0
                if only_stereo and not st2:
                    continue
                d = hamming(kf1["desc"][i1], kf2["desc"][i2])
                if d > 50 or d > best:
                    continue
                if not st1 and not st2:
                    dx = f32(ex - f32(k2["x"][i2]))
                    dy = f32(ey - f32(k2["y"][i2]))
                    if f32(f32(dx * dx) + f32(dy * dy)) < f32(f32(100) * f32(kf2["scale"][int(k2["octave"][i2])])):
                        continue
                if epi(i1, i2):
                    best, bi = d, i2
            if bi >= 0:
                m12[i1] = int(bi)
                nm += 1
                if check_ori:
                    hist[rot_bin(k1["angle"][i1], k2["angle"][bi])].append(i1)
    if check_ori:
        ind = three_maxima([len(h) for h in hist])
        for bn in range(30):
            if bn not in ind:
                for i1 in hist[bn]:
                    m12[i1] = -1
                    nm -= 1
    return np.array(m12, np.int32), nm
