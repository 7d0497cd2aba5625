"""Extract the rBRIEF sampling table bit_pattern_31_ from the reference source
text (src/ORBextractor.cc:236-494) into tests/golden/bit_pattern.npy.

The table is data (256 tests x {x0, y0, x1, y1}); this script reads the C
initializer as text, strips comments and evaluates every element as an
integer expression. The fork's element 96 reads `VX_FAILURE\\n -2`
(src/ORBextractor.cc:261-262); VX_FAILURE is OpenVX's vx_status_e value -1
(VX_FAILURE = -1 in the Khronos OpenVX 1.x headers, not vendored in the
reference), so that element is -3. Output: int8 array of shape (1024,) in the
reference's flat order. Run from the repo root:

    python tests/golden/make_pattern.py /root/reference/src/ORBextractor.cc
"""
from __future__ import annotations

import os
import re
import sys

import numpy as np

VX_FAILURE = -1  # OpenVX vx_status_e (VX_FAILURE = -1)


def parse(src_text: str) -> np.ndarray:
    m = re.search(r"static\s+int\s+bit_pattern_31_\s*\[\s*256\s*\*\s*4\s*\]\s*=\s*\{(.*?)\};", src_text, re.S)
    if not m:
        raise ValueError("bit_pattern_31_ initializer not found")
    body = re.sub(r"/\*.*?\*/", " ", m.group(1), flags=re.S)
    body = re.sub(r"//[^\n]*", " ", body)
    vals = []
    for tok in body.split(","):
        expr = " ".join(tok.split())
        if not expr:
            continue
        expr = expr.replace("VX_FAILURE", f"({VX_FAILURE})")
        if not re.fullmatch(r"[-+()\d\s]+", expr):
            raise ValueError(f"unexpected element {tok!r}")
        # integer expression of literals and +/- only: evaluate by tokens
        total, sign = 0, 1
        for t in re.findall(r"\d+|[-+]", expr.replace("(", " ").replace(")", " ")):
            if t == "-":
                sign = -sign
            elif t == "+":
                pass
            else:
                total += sign * int(t)
                sign = 1
        vals.append(total)
    if len(vals) != 1024:
        raise ValueError(f"expected 1024 elements, got {len(vals)}")
    return np.array(vals, np.int8)


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/src/ORBextractor.cc"
    with open(src, encoding="utf-8", errors="replace") as f:
        tbl = parse(f.read())
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bit_pattern.npy")
    np.save(out, tbl)
    print(f"wrote {out}: 1024 entries, [96] = {int(tbl[96])}")


if __name__ == "__main__":
    main()
