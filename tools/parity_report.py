"""Stage-by-stage parity report of the HIP extractor against the CPU oracle.

Usage: python tools/parity_report.py [seeds...]   (needs a gfx950 GPU)
Prints, per frame and level, whether pyramid, blur, FAST candidates and the
final keypoints/descriptors are bit-exact, and the first difference if not.
"""
import sys, os, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import orb_slam_cuda_amd as pkg
from oracle import oracle as O
from orb_slam_cuda_amd.synth import synth_frame


def report(seed, W=1241, H=376, nf=2000, **kw):
    ext = pkg.ORBextractor(nf, 1.2, 8, 20, 7, W, H, **kw)
    cfg = O.config(nfeatures=nf, width=W, height=H,
                   scale_mode=1 if kw.get("scale_mode") == "F" else 0,
                   pattern_mode=1 if kw.get("pattern") == "upstream" else 0)
    img = synth_frame(seed, W, H)
    t = time.time(); kp, desc = ext(img); tg = time.time() - t
    rkp, rdesc = O.extract(cfg, img)
    ok_all = True
    for l in range(8):
        g = ext.level_image(l); r = O.pyramid_level(cfg, img, l)
        gb = ext.level_image(l, blurred=True); rb = O.blur_level(cfg, img, l)
        fc = ext.fast_candidates(l); rc = O.fast_level(cfg, img, l)
        pyr_ok = g.shape == r.shape and np.array_equal(g, r)
        blur_ok = gb.shape == rb.shape and np.array_equal(gb, rb)
        fast_ok = len(fc) == len(rc) and all(np.array_equal(fc[f], rc[f]) for f in ("x", "y", "response"))
        lk = kp[kp["octave"] == l]; rl = rkp[rkp["octave"] == l]
        kp_ok = len(lk) == len(rl) and np.array_equal(lk.view(np.uint8), rl.view(np.uint8))
        ok_all &= pyr_ok and blur_ok and fast_ok and kp_ok
        line = f"seed {seed} L{l}: pyr {pyr_ok} blur {blur_ok} fast {fast_ok} ({len(fc)}/{len(rc)}) kps {kp_ok} ({len(lk)}/{len(rl)})"
        if not pyr_ok and g.shape == r.shape:
            d = np.argwhere(g != r); line += f" pyrdiff n={len(d)} first={d[:3].tolist()} g={g[tuple(d[0])]} r={r[tuple(d[0])]}"
        if not blur_ok and gb.shape == rb.shape:
            d = np.argwhere(gb != rb); line += f" blurdiff n={len(d)} first={d[:3].tolist()}"
        if not fast_ok:
            n = min(len(fc), len(rc)); bad = [i for i in range(n) if (fc[i]["x"], fc[i]["y"], fc[i]["response"]) != (rc[i]["x"], rc[i]["y"], rc[i]["response"])]
            line += f" fastdiff first={bad[:1]} g={fc[bad[0]] if bad else None} r={rc[bad[0]] if bad else None}"
        if not kp_ok and len(lk) == len(rl):
            for f in KP_FIELDS:
                if not np.array_equal(lk[f], rl[f]):
                    i = int(np.argmax(lk[f] != rl[f])); line += f" field {f} idx {i}: {lk[i]} vs {rl[i]};"
        print(line)
    dok = len(desc) == len(rdesc) and np.array_equal(desc, rdesc)
    if not dok and len(desc) == len(rdesc):
        rows = np.nonzero((desc != rdesc).any(1))[0]
        print(f"  desc mismatch rows {len(rows)} first {rows[:5]}")
    print(f"seed {seed}: total {len(kp)}/{len(rkp)} desc {dok} all {ok_all and dok} gpu_call {tg*1e3:.1f} ms")
    return ok_all and dok

KP_FIELDS = ("x", "y", "size", "angle", "response", "octave", "class_id")

if __name__ == "__main__":
    seeds = [int(s) for s in sys.argv[1:]] or [0, 1]
    ok = all([report(s) for s in seeds])
    ok &= report(3, 752, 480, 1000)
    sys.exit(0 if ok else 1)
