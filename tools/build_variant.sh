#!/bin/bash
# Build an experimental variant of the library with extra -D flags:
#   tools/build_variant.sh NAME "-DPM_DOWN_WAVES=7 ..."  ->  build_var/NAME/libpanman_amd.so
# Use it with PANMAN_AMD_LIB=build_var/NAME/libpanman_amd.so python bench.py ...
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; flags=${2:-}
out=build_var/$name
mkdir -p "$out"
objs=()
for f in panman_amd/csrc/*.cpp panman_amd/csrc/*.hip; do
  o=$out/$(basename "$f").o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $flags -x hip -c "$f" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o "$out/libpanman_amd.so" "${objs[@]}" -l:liblzma.so.5
echo "$out/libpanman_amd.so"
