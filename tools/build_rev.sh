#!/bin/bash
# Build the library of a git revision into build_var/NAME (A/B against the working tree):
#   tools/build_rev.sh NAME REV [extra -D flags] [PATCH.py]  ->  build_var/NAME/libpanman_amd.so
# (PATCH.py: edits the revision's csrc copy given as its argument, as in build_variant.sh)
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; rev=$2; flags=${3:-}; patch=${4:-}
out=build_var/$name
rm -rf "$out" && mkdir -p "$out/src"
git archive "$rev" panman_amd/csrc include | tar -x -C "$out/src"
src=$out/src/panman_amd/csrc
[ -n "$patch" ] && python3 "$patch" "$src"
objs=()
for f in $src/*.cpp $src/*.hip; do
  o=$out/$(basename "$f").o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -mllvm -amdgpu-atomic-optimizer-strategy=None -I"$out/src/include" $flags -x hip -c "$f" -o "$o" &
  objs+=("$o")
done
wait
id=$( (cat $(ls $src/*.cpp $src/*.hip $src/*.h | sort) $out/src/include/panman_gpu.h; echo "rev $rev $flags $patch") | sha256sum | cut -c1-16)
printf 'extern "C" const char* pm_build_id(void) { return "%s"; }\n' "$id" > "$out/pm_build_id.cpp"
g++ -O2 -fPIC -c "$out/pm_build_id.cpp" -o "$out/pm_build_id.o"
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o "$out/libpanman_amd.so" "${objs[@]}" "$out/pm_build_id.o" -l:liblzma.so.5
rm -rf "$out/src" "$out"/*.o
echo "$out/libpanman_amd.so"
