#!/bin/bash
# Build an experimental variant of the library with extra -D flags and, optionally, a source
# patch (a python script editing a copy of panman_amd/csrc given as its argument):
#   tools/build_variant.sh NAME "-DPM_DOWN_WAVES=7 ..." [PATCH.py]  ->  build_var/NAME/libpanman_amd.so
# Use it with PANMAN_AMD_LIB=build_var/NAME/libpanman_amd.so python bench.py ...
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; flags=${2:-}; patch=${3:-}
out=build_var/$name
mkdir -p "$out"
src=panman_amd/csrc
if [ -n "$patch" ]; then
  rm -rf "$out/src" "$out/include" && mkdir -p "$out/src" && cp -r panman_amd/csrc "$out/src/csrc" && cp -r include "$out/include"
  python3 "$patch" "$out/src/csrc"
  src=$out/src/csrc
fi
objs=()
for f in $src/*.cpp $src/*.hip; do
  o=$out/$(basename "$f").o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -mllvm -amdgpu-atomic-optimizer-strategy=None -I"$(pwd)/include" $flags -x hip -c "$f" -o "$o" &
  objs+=("$o")
done
wait
# the variant's own build id: its (possibly patched) sources, headers and compile flags, so
# PMC traffic stamped for another build is never reported against it
id=$( (cat $(ls $src/*.cpp $src/*.hip $src/*.h | sort) include/panman_gpu.h; echo "variant $flags") | sha256sum | cut -c1-16)
printf 'extern "C" const char* pm_build_id(void) { return "%s"; }\n' "$id" > "$out/pm_build_id.cpp"
g++ -O2 -fPIC -c "$out/pm_build_id.cpp" -o "$out/pm_build_id.o"
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o "$out/libpanman_amd.so" "${objs[@]}" "$out/pm_build_id.o" -l:liblzma.so.5
echo "$out/libpanman_amd.so"
