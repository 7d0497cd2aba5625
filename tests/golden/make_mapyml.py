"""Extract reference-held values from Examples/Monocular/map.yml, the map the
reference's own KeyFrame/MapPoint::write serialised (src/MapPoint.cc:424-491):

* the 775 MapPoint descriptors -> tests/golden/mapyml_descriptors.npy
  (775 x 32 uint8), real ORB descriptors for the Hamming pins;
* the 775 (mfMaxDistance, mfMinDistance) pairs -> tests/golden/mapyml_distances.npy
  (775 x 2 float32). MapPoint::UpdateNormalAndDepth writes
  mfMinDistance = mfMaxDistance / mvScaleFactors[nLevels-1]
  (src/MapPoint.cc:68-69, 372-373), so every pair pins the extractor's
  top-level scale factor of the run that wrote the map (tests/test_pins.py).

Run once in the build container (the reference is not on the GPU box); the
.npy files are committed. Text parsing only: nothing from the file is executed."""
import os, re, sys
import numpy as np

SRC = "/root/reference/Examples/Monocular/map.yml"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "mapyml_descriptors.npy")
OUT_DIST = os.path.join(HERE, "mapyml_distances.npy")


def descriptors(txt):
    rows = []
    for m in re.finditer(r"mDescriptor: !!opencv-matrix\s+rows: 1\s+cols: 32\s+dt: u\s+data: \[([^\]]*)\]", txt):
        v = [int(t) for t in m.group(1).replace("\n", " ").split(",")]
        assert len(v) == 32
        rows.append(v)
    return np.array(rows, np.uint8)


def distances(txt):
    """(max, min) per MapPoint, in file order; each point writes min then max (:489-490)."""
    pairs = re.findall(r"mfMinDistance: (\S+)\s+mfMaxDistance: (\S+)", txt)
    # the file holds floats printed as doubles: float32() of the text is the exact value written
    return np.array([(np.float32(float(mx)), np.float32(float(mn))) for mn, mx in pairs], np.float32)


def main():
    txt = open(SRC).read()
    a = descriptors(txt)
    np.save(OUT, a)
    print(a.shape, "->", OUT)
    d = distances(txt)
    assert len(d) == len(a)
    np.save(OUT_DIST, d)
    print(d.shape, "->", OUT_DIST)


if __name__ == "__main__":
    main()
