"""Seeded synthetic grayscale frames shaped like KITTI / EuRoC input.

KITTI and EuRoC images are not available offline, so the
benchmark and the parity tests run on synthetic scenes: a smooth gradient,
axis-aligned rectangles, ellipses and small textured blobs with uniform
intensities, plus uniform pixel noise. This gives a corner density in the
range of a real urban frame (thousands of FAST-7 corners at level 0).

A *sequence* is a random walk of a window over one larger canvas (integer
shifts in [-8, 8] per frame) with fresh noise per frame, so consecutive
frames share structure and the matchers find real correspondences.

All randomness comes from numpy's PCG64 (`np.random.default_rng(seed)`),
which is reproducible across platforms.
"""
from __future__ import annotations

import numpy as np

KITTI_WH = (1241, 376)
EUROC_WH = (752, 480)


def _paint_canvas(rng: np.random.Generator, W: int, H: int) -> np.ndarray:
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    base = rng.uniform(60, 190)
    gx, gy = rng.uniform(-0.08, 0.08, size=2)
    img = base + gx * (xx - W / 2) + gy * (yy - H / 2)
    area = W * H
    n_rect = max(8, int(90 * area / (1241 * 376)))
    n_ell = max(4, int(45 * area / (1241 * 376)))
    n_blob = max(4, int(60 * area / (1241 * 376)))
    for _ in range(n_rect):
        w = int(rng.integers(6, max(8, W // 6)))
        h = int(rng.integers(6, max(8, H // 4)))
        x0 = int(rng.integers(-w // 2, W))
        y0 = int(rng.integers(-h // 2, H))
        img[max(0, y0):max(0, y0 + h), max(0, x0):max(0, x0 + w)] = rng.uniform(0, 255)
    for _ in range(n_ell):
        cx, cy = rng.uniform(0, W), rng.uniform(0, H)
        a, b = rng.uniform(4, W / 10), rng.uniform(4, H / 6)
        th = rng.uniform(0, np.pi)
        x0, x1 = int(max(0, cx - a - b)), int(min(W, cx + a + b + 1))
        y0, y1 = int(max(0, cy - a - b)), int(min(H, cy + a + b + 1))
        if x1 <= x0 or y1 <= y0:
            continue
        sx = xx[y0:y1, x0:x1] - cx
        sy = yy[y0:y1, x0:x1] - cy
        u = sx * np.cos(th) + sy * np.sin(th)
        v = -sx * np.sin(th) + sy * np.cos(th)
        m = (u / a) ** 2 + (v / b) ** 2 <= 1.0
        img[y0:y1, x0:x1][m] = rng.uniform(0, 255)
    for _ in range(n_blob):
        # small checker / speckle patches: dense, strong corners (windows, foliage)
        bw, bh = int(rng.integers(10, 40)), int(rng.integers(10, 30))
        x0, y0 = int(rng.integers(0, max(1, W - bw))), int(rng.integers(0, max(1, H - bh)))
        cell = int(rng.integers(3, 8))
        lo, hi = sorted(rng.uniform(0, 255, size=2))
        pat = ((xx[y0:y0 + bh, x0:x0 + bw] // cell + yy[y0:y0 + bh, x0:x0 + bw] // cell) % 2)
        img[y0:y0 + bh, x0:x0 + bw] = np.where(pat > 0, hi, lo)
    return img


def synth_frame(seed: int, W: int = KITTI_WH[0], H: int = KITTI_WH[1]) -> np.ndarray:
    """One synthetic u8 frame (H x W, C-contiguous)."""
    rng = np.random.default_rng(seed)
    img = _paint_canvas(rng, W, H)
    img = img + rng.integers(-6, 7, size=img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


class SynthSequence:
    """A camera-like stream: a window random-walking over one canvas."""

    MARGIN = 96

    def __init__(self, seed: int, W: int = KITTI_WH[0], H: int = KITTI_WH[1]):
        self.W, self.H = W, H
        self.rng = np.random.default_rng(seed)
        M = self.MARGIN
        self.canvas = _paint_canvas(self.rng, W + 2 * M, H + 2 * M)
        self.ox, self.oy = M, M

    def shift(self) -> tuple[int, int]:
        dx, dy = (int(v) for v in self.rng.integers(-8, 9, size=2))
        M = self.MARGIN
        nx, ny = self.ox + dx, self.oy + dy
        # reflect the walk at the canvas edge
        if not 0 <= nx <= 2 * M:
            dx = -dx
        if not 0 <= ny <= 2 * M:
            dy = -dy
        self.ox += dx
        self.oy += dy
        return dx, dy

    def frame(self) -> np.ndarray:
        win = self.canvas[self.oy:self.oy + self.H, self.ox:self.ox + self.W]
        noisy = win + self.rng.integers(-6, 7, size=win.shape)
        return np.clip(np.rint(noisy), 0, 255).astype(np.uint8)

    def frames(self, n: int) -> np.ndarray:
        out = np.empty((n, self.H, self.W), np.uint8)
        for i in range(n):
            if i:
                self.shift()
            out[i] = self.frame()
        return out


class SynthStream:
    """A random-access synthetic sequence for splitting ONE sequence across
    ranks (bench.py --split-sequence): frame t is the window of the walk at t
    over one canvas with its own noise, so any rank renders its block (and the
    t-1 frame before it) without rendering the frames of the ranks before it.
    The walk (integer shifts in [-8, 8], reflected at the canvas edge, as
    SynthSequence) comes from its own generator, two draws per frame; the
    noise of frame t from default_rng((seed, t))."""

    MARGIN = SynthSequence.MARGIN

    def __init__(self, seed: int, W: int = KITTI_WH[0], H: int = KITTI_WH[1]):
        self.seed, self.W, self.H = seed, W, H
        self.canvas = _paint_canvas(np.random.default_rng(seed), W + 2 * self.MARGIN, H + 2 * self.MARGIN)
        self._walk = [(self.MARGIN, self.MARGIN)]
        self._wrng = np.random.default_rng((seed, 1 << 30))

    def origin(self, t: int) -> tuple[int, int]:
        M = self.MARGIN
        while len(self._walk) <= t:
            ox, oy = self._walk[-1]
            dx, dy = (int(v) for v in self._wrng.integers(-8, 9, size=2))
            if not 0 <= ox + dx <= 2 * M:
                dx = -dx
            if not 0 <= oy + dy <= 2 * M:
                dy = -dy
            self._walk.append((ox + dx, oy + dy))
        return self._walk[t]

    def frame(self, t: int) -> np.ndarray:
        ox, oy = self.origin(t)
        win = self.canvas[oy:oy + self.H, ox:ox + self.W]
        noisy = win + np.random.default_rng((self.seed, t)).integers(-6, 7, size=win.shape)
        return np.clip(np.rint(noisy), 0, 255).astype(np.uint8)

    def frames(self, idx) -> np.ndarray:
        idx = list(idx)
        out = np.empty((len(idx), self.H, self.W), np.uint8)
        for i, t in enumerate(idx):
            out[i] = self.frame(t)
        return out


def stereo_pair(seed: int, W: int = KITTI_WH[0], H: int = KITTI_WH[1]) -> tuple[np.ndarray, np.ndarray]:
    """Rectified left/right pair: the right image sees the scene shifted left
    by a disparity d in [5, 40] (a point at column u in the left image is at
    u - d in the right one), plus independent noise."""
    rng = np.random.default_rng(seed)
    canvas = _paint_canvas(rng, W + 48, H)
    disp = int(rng.integers(5, 41))
    left = canvas[:, :W]
    right = canvas[:, disp:disp + W]
    n = lambda a: np.clip(np.rint(a + rng.integers(-6, 7, size=a.shape)), 0, 255).astype(np.uint8)
    return n(left), n(right)


def synthetic_vocabulary(k: int = 10, L: int = 6, seed: int = 0, flip: float = 0.2,
                         scoring: int = 0, weighting: int = 0) -> dict:
    """A DBoW2-shaped ORB vocabulary (no ORBvoc.txt in this environment): a full
    k-ary tree of depth L in breadth-first file order (node 0 = root), each
    child's descriptor its parent's with a fraction `flip` of the bits flipped
    (a hierarchical clustering look-alike), leaves flagged as words with an
    idf-like weight log(N / n_i) > 0, inner nodes weight 0. Defaults follow
    ORB-SLAM2's ORBvoc.txt header (k 10, L 6, L1 scoring, TF-IDF)."""
    rng = np.random.default_rng(seed)
    counts = [k ** d for d in range(L + 1)]
    n = sum(counts)
    parent = np.zeros(n, np.int32)
    leaf = np.zeros(n, np.uint8)
    desc = np.zeros((n, 32), np.uint8)
    weight = np.zeros(n, np.float64)
    desc[0] = rng.integers(0, 256, 32, dtype=np.uint8)
    start = 1
    prev0 = 0
    for d in range(1, L + 1):
        m = counts[d]
        par = prev0 + np.arange(m) // k
        parent[start:start + m] = par
        bits = (rng.random((m, 256)) < flip).astype(np.uint8)
        desc[start:start + m] = desc[par] ^ np.packbits(bits, axis=1, bitorder="little")
        prev0 = start
        start += m
    nleaf = counts[L]
    leaf[n - nleaf:] = 1
    ni = rng.integers(1, 10000, nleaf)
    weight[n - nleaf:] = np.log(1e4 / ni) + 1e-3
    return dict(k=k, L=L, scoring=scoring, weighting=weighting, parent=parent, leaf=leaf, desc=desc,
                weight=weight)


def write_vocabulary_text(path: str, voc: dict) -> None:
    """DBoW2 text format (TemplatedVocabulary::saveToTextFile layout): header
    "k L scoring weighting", then one line per node after the root:
    "parent isLeaf d0 ... d31 weight" (weights written round-trip exact)."""
    with open(path, "w") as f:
        f.write(f"{voc['k']} {voc['L']} {voc['scoring']} {voc['weighting']}\n")
        for i in range(1, len(voc["parent"])):
            d = " ".join(str(int(b)) for b in voc["desc"][i])
            f.write(f"{int(voc['parent'][i])} {int(voc['leaf'][i])} {d} {float(voc['weight'][i])!r}\n")
