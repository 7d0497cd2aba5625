"""Extract the 775 MapPoint descriptors of the reference's Examples/Monocular/map.yml
(real ORB descriptors written by the reference's own KeyFrame/MapPoint::write,
src/MapPoint.cc:424) into tests/golden/mapyml_descriptors.npy (775 x 32 uint8).

Run once in the build container (the reference is not on the GPU box); the
.npy is committed. Text parsing only: nothing from the file is executed."""
import os, re, sys
import numpy as np

SRC = "/root/reference/Examples/Monocular/map.yml"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mapyml_descriptors.npy")

def main():
    txt = open(SRC).read()
    rows = []
    for m in re.finditer(r"mDescriptor: !!opencv-matrix\s+rows: 1\s+cols: 32\s+dt: u\s+data: \[([^\]]*)\]", txt):
        v = [int(t) for t in m.group(1).replace("\n", " ").split(",")]
        assert len(v) == 32
        rows.append(v)
    a = np.array(rows, np.uint8)
    np.save(OUT, a)
    print(a.shape, "->", OUT)

if __name__ == "__main__":
    main()
