set -e
for R in 1 2 4 8 16 32 64 128 256; do
  echo "rounds=$R"; ORBX_PROJ_ROUNDS=$R timeout -k 10 100 python tools/proj_timing.py 64
done
