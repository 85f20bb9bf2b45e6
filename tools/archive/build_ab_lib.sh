#!/bin/bash
# Builds monocular_depth_estimation_amd/libmde_hip_ab.so: the current objects
# with SRC (a csrc/*.hip file) taken from git revision REV (default HEAD), for
# tools/ab_lib.sh.   usage: tools/build_ab_lib.sh attn.hip [REV]
set -eu
cd "$(dirname "$0")/.."
src=$1; rev=${2:-HEAD}
make -C monocular_depth_estimation_amd/csrc -j8 >/dev/null
tmp=monocular_depth_estimation_amd/csrc/.ab_${src}
git show "$rev:monocular_depth_estimation_amd/csrc/$src" > "$tmp"
trap 'rm -f "$tmp"' EXIT
/opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -Iinclude -Wall -Wno-unused-function \
  -munsafe-fp-atomics -c -x hip "$tmp" -o build/ab_${src%.hip}.o
objs=$(ls build/csrc/*.o | grep -v "/${src%.hip}.o$")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o monocular_depth_estimation_amd/libmde_hip_ab.so $objs build/ab_${src%.hip}.o
echo "libmde_hip_ab.so: $src @ $rev"
