"""Host model of the sorted-key quadtree (orbx_quadtree.hip).

DistributeOctTree (src/ORBextractor.cc:889-1120) restated on keys sorted once
by their quadtree path code: a node box never depends on the data (roots from
nIni / hX, children from DivideNode's ceil halves, :831-887), so every node is
a contiguous range of the sorted keys and its children's ranges are found from
the codes alone. This script checks that restatement against the oracle's
orc_distribute on FAST keys of synthetic frames and prints the statistics that
size the kernel (keys, codes, bins, rounds, depths, sorted-round candidates).

    python tools/qt_model.py [--frames 4] [--config kitti|euroc|kitti14|intcatch1080]

Test infrastructure: it loads the oracle as the checker only.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from orb_slam_cuda_amd.synth import SynthSequence  # noqa: E402

CONFIGS = {
    "kitti": dict(nfeatures=2000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7, width=1241, height=376),
    "euroc": dict(nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7, width=752, height=480),
    "kitti14": dict(nfeatures=2000, scale_factor=1.2, nlevels=10, ini_th=17, min_th=7, width=1226, height=370),
    "intcatch1080": dict(nfeatures=2000, scale_factor=1.2, nlevels=3, ini_th=10, min_th=4, width=1920, height=1080),
}

f32 = np.float32


def c_round(v: float) -> int:
    return int(np.floor(abs(v) + 0.5)) * (1 if v >= 0 else -1)


def plan_level(boxW: int, boxH: int):
    """Root count, hX, root bits R, full depth D and the x / y path tables."""
    nIni = c_round(float(f32(boxW) / f32(boxH)))
    hX = f32(f32(boxW) / f32(nIni))
    R = max(1, int(np.ceil(np.log2(nIni)))) if nIni > 1 else 1
    D = (32 - R) // 2
    xs = np.zeros(boxW + 2, np.uint64)
    ys = np.zeros(boxH + 2, np.uint64)
    sep = True
    prev = None
    for x in range(boxW + 2):
        r = int(f32(x) / hX)
        a = int(f32(hX * f32(r)))
        c = int(f32(hX * f32(r + 1)))
        path = 0
        for j in range(D):
            mid = a + (c - a + 1) // 2
            bit = 1 if x >= mid else 0
            if bit:
                a = mid
            else:
                c = mid
            path |= bit << (D - 1 - j)
        code = r << (2 * D)
        for i in range(D):
            code |= ((path >> i) & 1) << (2 * i)
        if prev is not None and prev == code and x <= boxW:
            sep = False
        prev = code
        xs[x] = code
    a, c = 0, boxH
    prev = None
    for y in range(boxH + 2):
        a, c = 0, boxH
        path = 0
        for j in range(D):
            mid = a + (c - a + 1) // 2
            bit = 1 if y >= mid else 0
            if bit:
                a = mid
            else:
                c = mid
            path |= bit << (D - 1 - j)
        code = 0
        for i in range(D):
            code |= ((path >> i) & 1) << (2 * i + 1)
        if prev is not None and prev == code and y <= boxH:
            sep = False
        prev = code
        ys[y] = code
    return nIni, hX, R, D, xs, ys, sep


def distribute_sorted(keys, boxW, boxH, N, Dh_bins=4096, stats=None):
    """The kernel's algorithm, sequentially: returns the kept keys in list order."""
    nIni, hX, R, D, xs, ys, sep = plan_level(boxW, boxH)
    assert sep
    K = len(keys)
    x = keys["x"].astype(np.int64)
    y = keys["y"].astype(np.int64)
    code = (xs[x] | ys[y]).astype(np.uint64)
    order = np.argsort(code, kind="stable")
    sc = code[order]
    assert len(np.unique(sc)) == K, "codes not unique"

    def shift(d):
        return 2 * (D - d)

    def child_bounds(b, e, d):
        P = int(sc[b]) >> shift(d)
        res = []
        for q in (1, 2, 3):
            t = (P << 2) | q
            lo, hi = b, e
            while lo < hi:
                mid = (lo + hi) // 2
                if (int(sc[mid]) >> shift(d + 1)) < t:
                    lo = mid + 1
                else:
                    hi = mid
            res.append(lo)
        return res

    # roots: nodes in column order, empty ones erased
    lst = []  # (b, e, d, seq)
    for r in range(nIni):
        lo = int(np.searchsorted(sc, np.uint64(r << (2 * D)), "left"))
        hi = int(np.searchsorted(sc, np.uint64((r + 1) << (2 * D)), "left"))
        if hi > lo:
            lst.append((lo, hi, 0, 0))
    rounds = 0
    sorted_rounds = 0
    maxd = 0
    ncands = []
    finish = False
    sorted_phase = False
    prev_children = None
    while not finish:
        rounds += 1
        size = len(lst)
        if not sorted_phase:
            front = []  # children pushed to the front, most recent first
            rest = []
            nexp = 0
            stopped = False
            children_gt1 = []
            cur = len(lst)
            j = 0
            for idx, nd in enumerate(lst):
                if cur >= N:
                    rest.extend(lst[idx:])
                    stopped = True
                    break
                b, e, d, s = nd
                if e - b == 1:
                    rest.append(nd)
                    continue
                B = [b] + child_bounds(b, e, d) + [e]
                kids = []
                for q in range(4):
                    if B[q + 1] > B[q]:
                        kids.append((B[q], B[q + 1], d + 1, j * 4 + q))
                        maxd = max(maxd, d + 1)
                        if B[q + 1] - B[q] > 1:
                            nexp += 1
                            children_gt1.append(kids[-1])
                front = kids[::-1] + front
                cur += len(kids) - 1
                j += 1
            lst = front + rest
            if len(lst) >= N or len(lst) == size or stopped:
                finish = True
            elif len(lst) + 3 * nexp > N:
                sorted_phase = True
                prev_children = children_gt1
        else:
            sorted_rounds += 1
            cands = sorted(prev_children, key=lambda nd: ((nd[1] - nd[0]) << 16) | nd[3], reverse=True)
            ncands.append(len(cands))
            prev_children = []
            front = []
            split = set()
            cur = len(lst)
            for j, nd in enumerate(cands):
                b, e, d, s = nd
                B = [b] + child_bounds(b, e, d) + [e]
                kids = []
                for q in range(4):
                    if B[q + 1] > B[q]:
                        kids.append((B[q], B[q + 1], d + 1, j * 4 + q))
                        maxd = max(maxd, d + 1)
                        if B[q + 1] - B[q] > 1:
                            prev_children.append(kids[-1])
                front = kids[::-1] + front
                split.add((b, e, d))
                cur += len(kids) - 1
                if cur >= N:
                    break
            lst = front + [nd for nd in lst if (nd[0], nd[1], nd[2]) not in split]
            if len(lst) >= N or len(lst) == size:
                finish = True
    out = []
    for b, e, d, s in lst:
        idx = order[b:e]
        sc_ = keys["response"][idx]
        best = idx[int(np.argmax(sc_))]  # first max in sorted order ...
        m = sc_.max()
        best = int(np.min(idx[sc_ == m]))  # ... but ties go to the first in original order
        out.append(best)
    if stats is not None:
        bins = (sc >> np.uint64(2 * D - 2 * 5)).astype(np.int64)
        _, cnt = np.unique(bins, return_counts=True)
        stats.append(dict(K=K, nIni=nIni, R=R, D=D, rounds=rounds, sorted=sorted_rounds, maxd=maxd,
                          ncand=max(ncands) if ncands else 0, maxbin5=int(cnt.max()) if K else 0,
                          sum_bin2=int((cnt * cnt).sum()) if K else 0, nout=len(out)))
    return keys[np.array(out, np.int64)] if out else keys[:0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--config", default="kitti")
    a = ap.parse_args()
    c = CONFIGS[a.config]
    cfg = O.config(**c)
    info = O.level_info(cfg)
    frames = SynthSequence(3, c["width"], c["height"]).frames(a.frames)
    bad = 0
    for fi, img in enumerate(frames):
        for l in range(c["nlevels"]):
            w, h = int(info["w"][l]), int(info["h"][l])
            minX, maxX, minY, maxY = 16, w - 16, 16, h - 16
            keys = O.fast_level(cfg, img, l)
            N = int(info["nfeat"][l])
            ref = O.distribute(keys, minX, maxX, minY, maxY, N)
            st = []
            got = distribute_sorted(keys, maxX - minX, maxY - minY, N, stats=st)
            same = len(ref) == len(got) and np.array_equal(ref.view(np.uint8), got.view(np.uint8))
            bad += not same
            print(f"f{fi} L{l} {'OK ' if same else 'BAD'} {st[0]}")
    print("mismatches:", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
