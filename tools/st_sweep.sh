set -e
timeout -k 10 300 python -m pytest tests/test_gpu_stereo.py -x -q
for G in 2 4 8; do
  for S in 1 2 0; do
    ORBX_STEREO_GROUPS=$G ORBX_STEREO_STOP=$S timeout -k 10 60 python tools/stereo_timing.py 64
  done
done
