"""Timing experiment (A/B): leaf-plane loads non-temporal.  argv[2]: "up" (post-order code,
above struct DownArgs), "down" (below it) or "all"."""
import re
import sys
p = sys.argv[1] + "/pm_kernels.h"
which = sys.argv[2] if len(sys.argv) > 2 else "all"
s = open(p).read()
helper = """__device__ __forceinline__ uint4 load_stream(const uint4* p) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

"""
cut = s.index("struct DownArgs {")
up, down = s[:cut], s[cut:]
pat = re.compile(r"a\.leaf_planes\[([^\]]+)\]")
if which in ("up", "all"):
    up = pat.sub(r"load_stream(a.leaf_planes + (\1))", up)
if which in ("down", "all"):
    down = pat.sub(r"load_stream(a.leaf_planes + (\1))", down)
s = up + down
if "uint4 load_stream(" not in s:   # (the library has its own since the non-temporal record loads)
    anchor = "struct RecMask {"
    s = s.replace(anchor, helper + anchor, 1)
open(p, "w").write(s)
