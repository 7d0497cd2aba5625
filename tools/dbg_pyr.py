import sys, numpy as np
sys.path.insert(0, '.')
import orb_slam_cuda_amd as pkg
from oracle import oracle as O
from orb_slam_cuda_amd.synth import synth_frame
img = synth_frame(0)
ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, 1241, 376)
ext(img)
cfg = O.config()
g = ext.level_image(1).astype(int); r = O.pyramid_level(cfg, img, 1).astype(int)
bad = g != r
print("bad frac", bad.mean())
ys, xs = np.nonzero(bad)
print("by x%4", np.bincount(xs % 4, minlength=4), "by x//1024", np.bincount(xs // 1024))
print("rows with bad", np.unique(ys)[:20], "cols", np.unique(xs)[:40])
print("g row0", g[0, :16]); print("r row0", r[0, :16])
# is g a shifted version of r?
for s in range(-4, 5):
    print(s, np.mean(g[:, 8:-8] == np.roll(r, s, axis=1)[:, 8:-8]))
