"""Host<->device link rates on this box (pinned memory), for the host-streamed
leg: one C3 batch (64 KITTI frames) per copy.
  H2D 1D hipMemcpyAsync of the padded batch on 1 / 2 / 4 streams,
  H2D 2D DMA rectangle (unpadded 1241-byte rows -> 1280 pitch),
  H2D by a copy kernel reading pinned host memory (unpadded rows), 32..512 workgroups,
  D2H 1D hipMemcpyAsync of the batch's keypoint + descriptor block.
Prints one JSON line."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam_cuda_amd import _lib  # noqa: E402

L = _lib.lib()
vp = C.c_void_p
W, H, B, P = 1241, 376, 64, 1280
h_pad = _lib.HostArray((B, H, P), np.uint8)
h_raw = _lib.HostArray((B, H, W), np.uint8)
h_pad.a[:] = 7
h_raw.a[:] = 7
d_in = _lib.DeviceArray(B * H * P)
kpds = B * 2048 * 60
d_out = _lib.DeviceArray(kpds)
h_out = _lib.HostArray(kpds, np.uint8)
streams = [_lib.Stream() for _ in range(4)]
REPS = 30


def timed(fn, nbytes):
    for _ in range(3):
        fn()
    for s in streams:
        s.synchronize()
    t0 = time.perf_counter()
    for _ in range(REPS):
        fn()
    for s in streams:
        s.synchronize()
    dt = (time.perf_counter() - t0) / REPS
    return round(nbytes / dt / 1e9, 2)


out = {}
nb = B * H * P
for ns in (1, 2, 4):
    def f(ns=ns):
        for i in range(ns):
            lo, hi = i * nb // ns, (i + 1) * nb // ns
            _lib.check(L.orbx_memcpy_htod_async(vp(d_in.ptr + lo), vp(h_pad.ptr + lo), hi - lo, streams[i].s))
    out[f"h2d_1d_{ns}stream_GBps"] = timed(f, nb)


def f2():
    _lib.check(L.orbx_memcpy2d_htod_async(vp(d_in.ptr), P, vp(h_raw.ptr), W, W, B * H, streams[0].s))


out["h2d_2d_dma_unpadded_GBps"] = timed(f2, B * H * W)
for blocks in (32, 64, 128, 256, 512):
    def fk(blocks=blocks):
        _lib.check(L.orbx_copy2d_kernel_async(vp(d_in.ptr), P, vp(h_raw.ptr), W, W, B * H, blocks, streams[0].s))
    out[f"h2d_kernel_{blocks}wg_unpadded_GBps"] = timed(fk, B * H * W)
# correctness of the two unpadded paths
h_raw.a[:] = np.random.default_rng(0).integers(0, 256, (B, H, W), dtype=np.uint8)
for name, fn in (("dma", f2), ("kernel", lambda: L.orbx_copy2d_kernel_async(vp(d_in.ptr), P, vp(h_raw.ptr), W, W,
                                                                               B * H, 128, streams[0].s))):
    d_in.zero()
    fn()
    streams[0].synchronize()
    got = d_in.download((B, H, P), np.uint8)
    out[f"{name}_2d_exact"] = bool(np.array_equal(got[:, :, :W], h_raw.a))


def fd():
    _lib.check(L.orbx_memcpy_dtoh_async(vp(h_out.ptr), vp(d_out.ptr), kpds, streams[0].s))


out["d2h_1d_GBps"] = timed(fd, kpds)
print(json.dumps(out))
