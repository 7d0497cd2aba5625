"""The source-compatible C++ shim (shim/): ORB_SLAM2::ORBextractor,
ORBmatcher and ORBVocabulary re-implemented over include/orbx_c.h, compiled
with g++ against a minimal cv stub and linked to liborbx.so, driven by a small
C++ host that calls them as Tracking does (shim/host/driver.cc).

CPU: the shim builds, links and loads (no GPU call). GPU: the host's
ORBextractor::operator(), SearchForInitialization, Frame::ComputeBoW and both
SearchByBoW overloads give the oracle's results bit-exactly on KITTI-shaped
frames (reference interfaces: include/ORBextractor.h:75-197,
include/ORBmatcher.h:36-110)."""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "shim")
DRIVER = os.path.join(SHIM, "build", "orbx_shim_driver")
REF_H = "/root/reference/include"


def _build():
    subprocess.run(["make", "-s", "-C", SHIM], check=True)
    assert os.path.exists(DRIVER)


def test_shim_builds_and_links():
    _build()
    r = subprocess.run([DRIVER, "--version"], capture_output=True, text=True, check=True)
    assert r.stdout.startswith("orbx"), r.stdout
    ldd = subprocess.run(["ldd", DRIVER], capture_output=True, text=True, check=True).stdout
    assert "liborbx.so" in ldd and "not found" not in ldd, ldd


def _methods(text, cls):
    body = text[re.search(rf"class\s+{cls}\s*\{{", text).start():]
    return set(re.findall(r"\b(ORBextractor|ORBmatcher|operator\(\)|Get\w+|Search\w+|Fuse|DescriptorDistance)\s*\(", body))


@pytest.mark.skipif(not os.path.isdir(REF_H), reason="reference headers not present (GPU box)")
@pytest.mark.parametrize("name,cls", [("ORBextractor.h", "ORBextractor"), ("ORBmatcher.h", "ORBmatcher")])
def test_shim_declares_reference_surface(name, cls):
    ref = open(os.path.join(REF_H, name), encoding="utf-8", errors="replace").read()
    ours = open(os.path.join(SHIM, "include", name)).read()
    missing = _methods(ref, cls) - _methods(ours, cls)
    assert not missing, missing


@pytest.mark.gpu
def test_shim_host_matches_oracle(pkg, O, tmp_path):
    from orb_slam_cuda_amd.synth import SynthSequence, synthetic_vocabulary, write_vocabulary_text
    W, H, n = 1241, 376, 2
    assert os.path.exists(DRIVER), "build the shim first (make -C shim / __graft_entry__.build())"
    frames = SynthSequence(5, W, H).frames(n)
    fpath = tmp_path / "frames.u8"
    frames.tofile(fpath)
    voc = synthetic_vocabulary(6, 6, seed=3)
    vpath = tmp_path / "voc.txt"
    write_vocabulary_text(str(vpath), voc)
    out = tmp_path / "out"
    out.mkdir()
    r = subprocess.run([DRIVER, str(fpath), str(n), str(W), str(H), str(vpath), str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    cfg = O.config(nfeatures=2000, width=W, height=H)
    kps, descs = [], []
    for i in range(n):
        rkp, rdesc = O.extract(cfg, frames[i])
        kp = np.fromfile(out / f"kp{i}.bin", dtype=rkp.dtype)
        desc = np.fromfile(out / f"desc{i}.bin", dtype=np.uint8).reshape(-1, 32)
        assert len(kp) == len(rkp) > 1000
        assert np.array_equal(kp.view(np.uint8), rkp.view(np.uint8)), f"frame {i} keypoints"
        assert np.array_equal(desc, rdesc), f"frame {i} descriptors"
        # mvImagePyramid: headers over the pinned copy orbx_extract made beside its kernels
        for l in range(8):
            lvl = frames[i] if l == 0 else O.pyramid_level(cfg, frames[i], l)
            pyr = np.fromfile(out / f"pyr{l}_{i}.bin", dtype=np.uint8).reshape(lvl.shape)
            assert np.array_equal(pyr, lvl), f"frame {i} mvImagePyramid[{l}]"
        kps.append(rkp)
        descs.append(rdesc)
    (k1, k2), (d1, d2) = kps, descs
    # SearchForInitialization(F1, F2, mvbPrevMatched = F1 keypoints, 100), ratio 0.9
    rec = np.fromfile(out / "init.bin", dtype=np.int32)
    prev = np.fromfile(out / "init_prev.bin", dtype=np.float32).reshape(-1, 2)
    r12, rnm, rprev = O.search_for_initialization(k1, d1, k2, d2, (0, W, 0, H), np.stack([k1["x"], k1["y"]], 1),
                                                  100, 0.9, True)
    assert rec[0] == rnm > 50 and np.array_equal(rec[1:], r12) and np.array_equal(prev, rprev)
    assert np.fromfile(out / "dist.bin", dtype=np.int32)[0] == O.descriptor_distance(d1[0], d2[0])
    # ComputeBoW + SearchByBoW: MapPoints on features i % 4 != 3, bad when i % 7 == 5
    fv = []
    for d in (d1, d2):
        t = O.voc_transform(voc, d, 4)
        fv.append((t["fv_nodes"], t["fv_off"], t["fv_idx"]))
    good = lambda k: np.array([(i % 4 != 3) and (i % 7 != 5) for i in range(len(k))], np.uint8)
    rout, rnm = O.search_by_bow(d1, k1["angle"], good(k1), fv[0], d2, k2["angle"], np.ones(len(k2), np.uint8), fv[1],
                                0.7, True, False)
    got = np.fromfile(out / "bow_kf_f.bin", dtype=np.int32)
    assert got[0] == rnm > 20 and np.array_equal(got[1:], rout)
    rout, rnm = O.search_by_bow(d1, k1["angle"], good(k1), fv[0], d2, k2["angle"], good(k2), fv[1], 0.75, True, True)
    got = np.fromfile(out / "bow_kf_kf.bin", dtype=np.int32)
    assert got[0] == rnm > 20 and np.array_equal(got[1:], rout)


# ------------------------------------------------------------ scene mode
SCENES = [("local_map", dict(seed=1)), ("local_map", dict(seed=2, th=1.0, ratio=0.9, stereo=False)),
          ("last_frame", dict(seed=1)), ("last_frame", dict(seed=2, stereo=False, motion="none")),
          ("keyframe", dict(seed=1)), ("keyframe", dict(seed=2, th=3.0, orb_dist=64)),
          ("sim3", dict(seed=1)), ("sim3", dict(seed=2, th=5, s=0.7)),
          ("fuse", dict(seed=1)), ("fuse", dict(seed=2, th=5.0)),
          ("fuse_sim3", dict(seed=1)), ("sim3_match", dict(seed=1)), ("sim3_match", dict(seed=2, s12=1.08)),
          ("triangulation", dict(seed=1)), ("triangulation", dict(seed=2, only_stereo=True)),
          ("bow", dict(seed=1)), ("bow", dict(seed=3, ratio=0.75))]


@pytest.mark.gpu
@pytest.mark.parametrize("op,kw", SCENES, ids=[f"{o}-{i}" for i, (o, _) in enumerate(SCENES)])
def test_shim_matcher_methods_match_oracle(pkg, O, tmp_path, op, kw):
    """Every ORBmatcher method through the compiled drop-in shim, called on
    reference-typed Frames / KeyFrames / MapPoints as Tracking, LocalMapping
    and LoopClosing call it (shim/host/scene.cc), against the oracle's result
    translated into the pointer state the reference leaves (tests/shimscene.py)."""
    import shimscene
    assert os.path.exists(DRIVER), "build the shim first (make -C shim / __graft_entry__.build())"
    recs, want = getattr(shimscene, op)(O, **kw)
    scene, out = tmp_path / "scene.bin", tmp_path / "out.bin"
    shimscene.write_scene(scene, recs)
    r = subprocess.run([DRIVER, "--scene", str(scene), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(out, dtype=np.int32)
    assert got[0] == want[0], (op, got[0], want[0])
    assert np.array_equal(got, want), (op, np.nonzero(got[:len(want)] != want[:len(got)])[0][:10])
    assert want[0] > 20  # the scene exercises the method


_STEREO_REFS = {}


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [0, 1])
def test_shim_stereo_frame_matches_oracle(pkg, O, tmp_path, threads):
    """The stereo Frame constructor through the shim over 16 stereo pairs, against
    the oracle's extraction + stereo matching. threads=0: the drop-in body
    Frame::ExtractStereo (both extractions and ComputeStereoMatches with one
    device round trip, orbm_stereo_frame). threads=1 (ORBX_STEREO_THREADS=1): the
    reference's structure, two ORBextractors driven from two std::threads per
    Frame (src/Frame.cc:77-80), then Frame::ComputeStereoMatches (:465-639) over
    orbm_compute_stereo_matches_last; its first Frame also races the two
    handles' first launches (the per-device BRIEF table upload)."""
    from concurrent.futures import ThreadPoolExecutor

    from orb_slam_cuda_amd.synth import stereo_pair
    assert os.path.exists(DRIVER)
    W, H, bf, n = 1241, 376, 0.54 * 718.856, 16
    pairs = [stereo_pair(21 + i, W, H) for i in range(n)]
    lp, rp = tmp_path / "l.u8", tmp_path / "r.u8"
    np.ascontiguousarray(np.stack([p[0] for p in pairs])).tofile(lp)
    np.ascontiguousarray(np.stack([p[1] for p in pairs])).tofile(rp)
    env = dict(os.environ, ORBX_STEREO_THREADS=str(threads))
    r = subprocess.run([DRIVER, "--stereo", str(lp), str(rp), str(n), str(W), str(H), repr(bf), str(tmp_path)],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    cfg = O.config(nfeatures=2000, width=W, height=H)
    info = O.level_info(cfg)
    mb = np.fromfile(tmp_path / "mb.bin", dtype=np.float32)[0]
    assert mb == np.float32(bf) / np.float32(718.856)

    def ref(i):
        if i in _STEREO_REFS:
            return _STEREO_REFS[i]
        L, R = pairs[i]
        kl, dl = O.extract(cfg, L)
        kr, dr = O.extract(cfg, R)
        ru, rd, rk = O.compute_stereo_matches(kl, dl, kr, dr, O.pyramid(cfg, L), O.pyramid(cfg, R), info["scale"],
                                              info["inv_scale"], mb, np.float32(bf))
        _STEREO_REFS[i] = (kl, dl, kr, dr, ru, rd, rk)
        return _STEREO_REFS[i]

    with ThreadPoolExecutor(8) as ex:
        refs = list(ex.map(ref, range(n)))
    for i, (kl, dl, kr, dr, ru, rd, rk) in enumerate(refs):
        got = lambda name, dt: np.fromfile(tmp_path / f"{name}{i}.bin", dtype=dt)
        assert np.array_equal(got("kpL", kl.dtype).view(np.uint8), kl.view(np.uint8)), i
        assert np.array_equal(got("kpR", kr.dtype).view(np.uint8), kr.view(np.uint8)), i
        assert np.array_equal(got("descL", np.uint8).reshape(-1, 32), dl), i
        assert np.array_equal(got("descR", np.uint8).reshape(-1, 32), dr), i
        u, d = got("uright", np.float32), got("depth", np.float32)
        assert np.array_equal(u, ru) and np.array_equal(d, rd) and rk > 100, i


def test_shim_defines_every_reference_method():
    """No ORBmatcher method of the reference header is declared without a
    definition in the shim (each appears as ORBmatcher::Name in src/ORBmatcher.cc)."""
    text = open(os.path.join(SHIM, "include", "ORBmatcher.h")).read()
    body = open(os.path.join(SHIM, "src", "ORBmatcher.cc")).read()
    declared = set(re.findall(r"\b(Search\w+|Fuse|DescriptorDistance)\s*\(", text))
    for name in declared:
        assert f"ORBmatcher::{name}(" in body, name
    # overload counts: 4 SearchByProjection, 2 SearchByBoW, 2 Fuse
    for name, k in (("SearchByProjection", 4), ("SearchByBoW", 2), ("Fuse", 2)):
        assert body.count(f"int ORBmatcher::{name}(") == k, name
    assert "void Frame::ComputeStereoMatches()" in open(os.path.join(SHIM, "src", "Frame.cc")).read()


@pytest.mark.gpu
@pytest.mark.parametrize("mode,pattern", [("F", "fork"), ("U", "upstream")])
def test_shim_extractor_modes_from_environment(pkg, O, tmp_path, mode, pattern):
    """The shim's ORBextractor reads ORBX_SCALE_MODE / ORBX_PATTERN / ORBX_DEVICE
    once in its constructor (shim/src/ORBextractor.cc): mode F (the fork's
    buildGraph scale override, src/ORBextractor.cc:674-680) and the upstream
    pattern through operator() against the oracle in the same modes."""
    from orb_slam_cuda_amd.synth import SynthSequence
    W, H, n = 1241, 376, 1
    frames = SynthSequence(9, W, H).frames(n)
    fpath = tmp_path / "frames.u8"
    frames.tofile(fpath)
    out = tmp_path / "out"
    out.mkdir()
    env = dict(os.environ, ORBX_SCALE_MODE=mode, ORBX_PATTERN=pattern, ORBX_DEVICE="0")
    r = subprocess.run([DRIVER, str(fpath), str(n), str(W), str(H), "-", str(out)], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    cfg = O.config(nfeatures=2000, width=W, height=H, scale_mode=1 if mode == "F" else 0,
                   pattern_mode=1 if pattern == "upstream" else 0)
    rkp, rdesc = O.extract(cfg, frames[0])
    kp = np.fromfile(out / "kp0.bin", dtype=rkp.dtype)
    desc = np.fromfile(out / "desc0.bin", dtype=np.uint8).reshape(-1, 32)
    assert len(kp) == len(rkp) > 1000
    assert np.array_equal(kp.view(np.uint8), rkp.view(np.uint8)) and np.array_equal(desc, rdesc)
    if mode == "F":  # level sizes differ from mode U: the override really took effect
        lvl = O.pyramid_level(cfg, frames[0], 1)
        assert lvl.shape != O.pyramid_level(O.config(), frames[0], 1).shape


@pytest.mark.gpu
def test_shim_extractor_without_camera_size(pkg, O, tmp_path):
    """Tracking passes Camera.width/height = 0 for the reference's mono yamls
    (Examples/Monocular/KITTI00-02.yaml has neither key, src/Tracking.cc:124-133):
    the extractor constructs, its scale getters return the 1.2^l tables before
    the first call (the Frame ctor reads them first, src/Frame.cc:181-190), and
    the first 1241x376 frame extracts bit-exact against the oracle."""
    from orb_slam_cuda_amd.synth import SynthSequence
    W, H, n = 1241, 376, 2
    frames = SynthSequence(13, W, H).frames(n)
    fpath = tmp_path / "frames.u8"
    frames.tofile(fpath)
    out = tmp_path / "out"
    out.mkdir()
    env = dict(os.environ, ORBX_DRIVER_CTOR_WH="0")
    r = subprocess.run([DRIVER, str(fpath), str(n), str(W), str(H), "-", str(out)], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    cfg = O.config(nfeatures=2000, width=W, height=H)
    info = O.level_info(cfg)
    sc = np.fromfile(out / "scales_pre.bin", dtype=np.float32).reshape(4, 8)
    for row, key in zip(sc, ("scale", "inv_scale", "sigma2", "inv_sigma2")):
        assert np.array_equal(row, info[key]), key
    for i in range(n):
        rkp, rdesc = O.extract(cfg, frames[i])
        kp = np.fromfile(out / f"kp{i}.bin", dtype=rkp.dtype)
        desc = np.fromfile(out / f"desc{i}.bin", dtype=np.uint8).reshape(-1, 32)
        assert len(kp) == len(rkp) > 1000
        assert np.array_equal(kp.view(np.uint8), rkp.view(np.uint8)) and np.array_equal(desc, rdesc)


def test_shim_rejects_unknown_scale_mode(tmp_path):
    _build()
    frames = np.zeros((1, 64, 64), np.uint8)
    fpath = tmp_path / "f.u8"
    frames.tofile(fpath)
    env = dict(os.environ, ORBX_SCALE_MODE="Q")
    r = subprocess.run([DRIVER, str(fpath), "1", "64", "64", "-", str(tmp_path)], capture_output=True, text=True,
                       timeout=60, env=env)
    assert r.returncode != 0 and "ORBX_SCALE_MODE" in r.stderr


def test_shim_gettime_tracking_usage(tmp_path):
    """Tracking's own use of the header's timing records (src/Tracking.cc:290,
    172-190: GetTime(times, n, name, -1) scopes, then a loop over times_t)
    compiles against the shim's ORBextractor.h and runs on the CPU."""
    _build()
    src = tmp_path / "t.cc"
    src.write_text(
        '#include <cstdio>\n#include "ORBextractor.h"\nusing namespace ORB_SLAM2;\n'
        'int main() { std::vector<times_t> times; int n = 0;\n'
        '  for (int k = 0; k < 3; ++k) { GetTime tmp(times, n++, "Track", -1); }\n'
        '  for (times_t t : times) printf("%d;%s;%d;%d\\n", t.frame, t.name.c_str(), t.level, t.time >= 0);\n'
        '  return 0; }\n')
    exe = tmp_path / "t"
    objs = [os.path.join(SHIM, "build", "src", "ORBextractor.o")]
    subprocess.run(["g++", "-std=c++14", "-pthread", "-I", os.path.join(SHIM, "include"), "-I",
                    os.path.join(SHIM, "cv"), "-I", os.path.join(ROOT, "include"), str(src), *objs,
                    "-L", os.path.join(ROOT, "orb_slam_cuda_amd"), "-lorbx",
                    f"-Wl,-rpath,{os.path.join(ROOT, 'orb_slam_cuda_amd')}", "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    assert out.split() == ["0;Track;-1;1", "1;Track;-1;1", "2;Track;-1;1"]


@pytest.mark.gpu
def test_shim_times_csv(pkg, tmp_path):
    """ORBX_TIMING=1: every operator() call records the device stage times under
    the reference's GetTime names (in the stages' launch order) plus "Total
    Time ORB extraction", and the
    destructor appends them to ./times.csv in the reference's layout
    (src/ORBextractor.cc:800-820): '#Frame;Name Processing function;Level;Time
    spent (ns);Time spent (ms)' then 'frame;name;level;ns;ms;' rows."""
    from orb_slam_cuda_amd.synth import SynthSequence
    W, H, n = 1241, 376, 3
    frames = SynthSequence(5, W, H).frames(n)
    fpath = tmp_path / "frames.u8"
    frames.tofile(fpath)
    out = tmp_path / "out"
    out.mkdir()
    env = dict(os.environ, ORBX_TIMING="1")
    r = subprocess.run([DRIVER, str(fpath), str(n), str(W), str(H), "-", str(out)], capture_output=True, text=True,
                       timeout=120, env=env, cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    assert "Avg computed frame ORB:" in r.stdout
    lines = (tmp_path / "times.csv").read_text().splitlines()
    assert lines[0] == "#Frame;Name Processing function;Level;Time spent (ns);Time spent (ms)"
    rows = [l.split(";") for l in lines[1:]]
    # the stage records in launch order (orbx_get_stage_order), then the total
    label = {"pyramid": "Pyramid/Resize", "blur": "Gaussian Blur", "fast_grid": "FAST+Grid", "quadtree": "Make quadtree",
             "orient_brief": "Compute angle+ORB descriptor+scale"}
    from orb_slam_cuda_amd import _lib
    names = [label[s] for s in _lib.stage_order()] + ["Total Time ORB extraction"]
    assert len(rows) == n * len(names)
    for k, row in enumerate(rows):
        assert len(row) == 6 and row[5] == ""
        assert int(row[0]) == k // len(names) and row[1] == names[k % len(names)] and row[2] == "-1"
        ns, ms = int(row[3]), float(row[4])
        assert ns > 0 and abs(ms - ns / 1e6) <= 1e-3 * max(1.0, ms)
    # stages of one call fit inside its host total
    for f in range(n):
        st = rows[f * len(names):(f + 1) * len(names)]
        assert sum(int(r[3]) for r in st[:-1]) <= int(st[-1][3])
