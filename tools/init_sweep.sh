set -e
for S in 1 2 3 0; do ORBX_INIT_STOP=$S timeout -k 10 100 python tools/init_timing.py 64; done
WHICH=hamming timeout -k 10 100 python tools/init_timing.py 64
