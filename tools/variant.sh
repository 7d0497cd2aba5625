#!/bin/bash
# Build an A/B variant of liborbx.so: one source recompiled with extra -D flags,
# linked with the other objects of the normal build.
#   tools/variant.sh <name> <source.hip> [-DNAME=VALUE ...]
# -> orb_slam_cuda_amd/variants/liborbx_<name>.so, loaded with ORBX_LIB_VARIANT=<name>
# (built with -DORBX_DIAG: bench.py refuses variants unless --allow-diag, and stamps the line)
set -e
name=$1; src=$2; shift 2
cd "$(dirname "$0")/../orb_slam_cuda_amd/csrc"
make -s
mkdir -p build/var ../variants
obj=build/var/${name}_$(basename "$src" .hip).o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../../include -DORBX_DIAG "$@" -c "$src" -o "$obj"
objs=$(ls build/*.o | grep -v "build/$(basename "$src" .hip).o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../variants/liborbx_${name}.so $objs "$obj"
echo "built variants/liborbx_${name}.so"
