"""Row counts of the band pyramid with and without a blur halo (DESIGN.md §6,
round 5): for the KITTI plan's bands (R rows of the last level each), the
rows of every level a band must compute when it only feeds the next level
(halo 0, the shipped plan) and when it must also blur its own rows in LDS
(halo 3 at every level, which cascades: each halo row of level l+1 needs its
INTER_LINEAR source rows of level l). Same row tables as plan_band_pyramid
(orbx_host.hip): OpenCV 3.x INTER_LINEAR source rows per output row.
Usage: python tools/halo_cascade.py [R]"""
import math
import sys

import numpy as np

W, H, L, R = 1241, 376, 8, int(sys.argv[1]) if len(sys.argv) > 1 else 5
lw = [int(np.rint(np.float32(W) * np.float32(1.0 / 1.2 ** l))) for l in range(L)]
lh = [int(np.rint(np.float32(H) * np.float32(1.0 / 1.2 ** l))) for l in range(L)]


def ytab(sh, dh):
    sc = sh / dh
    out = []
    for dy in range(dh):
        sy = int(math.floor(np.float32((dy + 0.5) * sc - 0.5)))
        out.append((min(max(sy, 0), sh - 1), min(max(sy + 1, 0), sh - 1)))
    return out


yt = [None] + [ytab(lh[l - 1], lh[l]) for l in range(1, L)]


def rows(halo):
    nb = (lh[-1] + R - 1) // R
    tot = [0] * L
    for b in range(nb):
        lo, hi = [0] * L, [0] * L
        lo[-1], hi[-1] = max(0, b * R - halo), min(min((b + 1) * R, lh[-1]) - 1 + halo, lh[-1] - 1)
        for l in range(L - 2, -1, -1):
            lo[l] = max(0, yt[l + 1][lo[l + 1]][0] - halo)
            hi[l] = min(lh[l] - 1, yt[l + 1][hi[l + 1]][1] + halo)
        for l in range(L):
            tot[l] += hi[l] - lo[l] + 1
    return nb, tot


for halo in (0, 3):
    nb, tot = rows(halo)
    px = sum(tot[l] * lw[l] for l in range(1, L))
    print(f"halo {halo}: {nb} bands, rows per level {tot}, level-0 rows staged {tot[0]}, "
          f"computed px of levels 1..{L - 1} {px} (the levels hold {sum(lh[l] * lw[l] for l in range(1, L))})")
