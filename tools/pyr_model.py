"""Host-side model of the band pyramid's tilings (orbx_host.hip
plan_band_pyramid / plan_pyr_cols restated): per (bands, column tiles) the
worst tile's pixel count and row-loop iterations, for fitting the plan
picker's cost rule against tools/pyr_plans.py timings.
Usage: python3 tools/pyr_model.py [W H NLEVELS SCALE]"""
import math
import sys

W, H, L = (int(a) for a in (sys.argv[1:4] if len(sys.argv) >= 4 else (1241, 376, 8)))
SF = float(sys.argv[4]) if len(sys.argv) >= 5 else 1.2
T = 512  # threads per workgroup

sizes = []
for l in range(L):
    inv = 1.0 / SF ** l
    sizes.append((int(round(W * inv)), int(round(H * inv))))


def src(sw, dw):
    """per output index: (lo, hi) source indices of INTER_LINEAR (2x: area)"""
    scale = sw / dw
    if abs(scale - 2.0) < 1e-12:
        return [(2 * d, 2 * d + 1) for d in range(dw)]
    out = []
    for d in range(dw):
        f = (d + 0.5) * scale - 0.5
        s = math.floor(f)
        s = max(s, 0)
        s = min(s, sw - 1)
        out.append((s, min(s + 1, sw)))
    return out


xs = [None] + [src(sizes[l - 1][0], sizes[l][0]) for l in range(1, L)]
ys = [None] + [src(sizes[l - 1][1], sizes[l][1]) for l in range(1, L)]


def ranges(n_last, parts, tabs, dims, even):
    lo = [[0] * L for _ in range(parts)]
    chi = [[0] * L for _ in range(parts)]
    for c in range(parts):
        a = c * n_last // parts
        b = (c + 1) * n_last // parts
        if even:
            a &= ~1
            b = b & ~1 if c + 1 < parts else b
        lo[c][L - 1] = a
        chi[c][L - 1] = b - 1
    for l in range(L - 2, -1, -1):
        for c in range(parts):
            v = 0 if c == 0 else tabs[l + 1][min(lo[c][l + 1], dims[l + 1] - 1)][0]
            lo[c][l] = v & ~1 if even else v
    for l in range(L - 2, -1, -1):
        for c in range(parts):
            own_hi = lo[c + 1][l] - 1 if c + 1 < parts else dims[l] - 1
            chi[c][l] = max(tabs[l + 1][min(chi[c][l + 1], dims[l + 1] - 1)][1], own_hi if l > 0 else 0)
    return lo, chi


def plan(nb, nct):
    HL = sizes[L - 1][1]
    R = -(-HL // nb)
    nb = -(-HL // R)
    rl, rc = ranges(HL, nb, ys, [s[1] for s in sizes], False)
    # rows: bands of R rows (the kernel's planner uses b*R, not b*HL//nb)
    for b in range(nb):
        rl[b][L - 1] = b * R
        rc[b][L - 1] = min((b + 1) * R, HL) - 1
    for l in range(L - 2, -1, -1):
        for b in range(nb):
            rl[b][l] = 0 if b == 0 else ys[l + 1][rl[b][l + 1]][0]
    for l in range(L - 2, -1, -1):
        for b in range(nb):
            own_hi = rl[b + 1][l] - 1 if b + 1 < nb else sizes[l][1] - 1
            rc[b][l] = max(ys[l + 1][rc[b][l + 1]][1], own_hi if l > 0 else 0)
    cl, cc = ranges(sizes[L - 1][0], nct, xs, [s[0] for s in sizes], True)
    worst_px = worst_it = 0
    tot_px = 0
    for b in range(nb):
        for c in range(nct):
            px = it = 0
            for l in range(L):
                rows = rc[b][l] - rl[b][l] + 1
                wt = cc[c][l] - cl[c][l] + 1
                px += rows * wt
                if l >= 1:
                    G = (wt + 7) // 8
                    it += -(-rows // (T // G))
            worst_px = max(worst_px, px)
            worst_it = max(worst_it, it)
            tot_px += px
    return nb, worst_px, worst_it, tot_px


if __name__ == "__main__":
    for nct in (1, 2, 4):
        for nb in (10, 11, 12, 14, 15, 18, 21, 27, 35, 53):
            n, px, it, tot = plan(nb, nct)
            print(f"{n}:{nct} worst_px {px} worst_iters {it} total_px/frame {tot}")
