#!/bin/bash
# Build a variant of libciruela_amd.so with extra compile flags into
# abtest/NAME.so (for tools/ab_lib.py / ab_quad.py A/B runs on the box).
# Usage: tools/build_variant.sh NAME [-DFLAG=VALUE ...]
set -eu
cd "$(dirname "$0")/.."
name=$1
shift
obj=build/variant_$name
mkdir -p "$obj" abtest
flags="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Iinclude -Iciruela_amd/csrc"
for f in kernels order; do
  /opt/rocm/bin/hipcc $flags --offload-arch=gfx950 -mcode-object-version=5 "$@" \
    -c ciruela_amd/csrc/$f.hip -o "$obj/$f.o" &
done
for f in runtime dirsig scan registry blake2b_host sha512_host; do
  /opt/rocm/bin/hipcc $flags -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include "$@" \
    -c ciruela_amd/csrc/$f.cpp -o "$obj/$f.o" &
done
wait
/opt/rocm/bin/hipcc $flags --offload-arch=gfx950 -mcode-object-version=5 -shared \
  -o "abtest/$name.so" "$obj"/*.o -lpthread
echo "abtest/$name.so"
