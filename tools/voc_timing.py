"""Times orbv_transform_batch alone on a resident batch of extracted descriptors
(tuning aid). Usage: python tools/voc_timing.py [frames]; env ORBX_VOC_STOP=1 = descend only."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import orb_slam_cuda_amd as pkg  # noqa: E402
from orb_slam_cuda_amd import _lib  # noqa: E402
from orb_slam_cuda_amd.synth import SynthSequence, synthetic_vocabulary  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
W, H = 1241, 376
voc = pkg.ORBVocabulary.from_arrays(synthetic_vocabulary(10, 6, seed=1))
frames = np.ascontiguousarray(SynthSequence(3, W, H).frames(B))
ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H, max_batch=B)
cap = ext.frame_capacity
d_in = _lib.DeviceArray(frames.nbytes)
d_in.upload(frames)
d_kp, d_desc, d_n = _lib.DeviceArray(B * cap * 28), _lib.DeviceArray(B * cap * 32), _lib.DeviceArray(4 * B)
s = _lib.Stream()
ext.extract_batch_device(d_in.ptr, B, H * W, W, d_kp.ptr, d_desc.ptr, d_n.ptr, s)
outs = [_lib.DeviceArray(B * cap * 8) for _ in range(5)] + [_lib.DeviceArray(B * (cap + 1) * 4)] + \
       [_lib.DeviceArray(B * 4) for _ in range(2)] + [_lib.DeviceArray(B * cap * 8) for _ in range(3)]
L = _lib.lib()
v = C.c_void_p


def run():
    _lib.check(L.orbv_transform_batch(voc.handle, v(d_desc.ptr), cap * 32, v(d_n.ptr), B, cap, 4, v(outs[0].ptr),
                                      v(outs[1].ptr), v(outs[6].ptr), v(outs[2].ptr), v(outs[5].ptr), v(outs[3].ptr),
                                      v(outs[7].ptr), v(outs[8].ptr), v(outs[9].ptr), v(outs[10].ptr), s.s),
               vocabulary=True)


for _ in range(3):
    run()
e0, e1 = _lib.Event(), _lib.Event()
N = 20
e0.record(s)
for _ in range(N):
    run()
e1.record(s)
s.synchronize()
print(f"frames={B} stop={os.environ.get('ORBX_VOC_STOP', '0')} ms_per_call={e0.elapsed_ms(e1) / N:.4f} "
      f"words_mean={outs[6].download(B, np.int32).mean():.1f}")
