"""Timing experiment (A/B): the pre-order's mutation-record stores non-temporal."""
import sys
p = sys.argv[1] + "/pm_kernels.h"
s = open(p).read()
helper = """__device__ __forceinline__ void store_rec_nt(pm_mut* p, uint32_t node, uint32_t info) {
    __builtin_nontemporal_store(((uint64_t)info << 32) | node, reinterpret_cast<uint64_t*>(p));
}

"""
anchor = "// One round of a flush"
assert anchor in s
s = s.replace(anchor, helper + anchor, 1)
pairs = [
    ("            if ((int64_t)p < cap) out[p] = pm_mut{node, ((site0 + (uint32_t)b) << 8) | rec_low(e1.x, e1.y, e1.z, e1.w, pz, b)};",
     "            if ((int64_t)p < cap) store_rec_nt(out + p, node, ((site0 + (uint32_t)b) << 8) | rec_low(e1.x, e1.y, e1.z, e1.w, pz, b));"),
    ("                if ((int64_t)q < cap) out[q] = pm_mut{hn, ((hs + (uint32_t)bit) << 8) | rec_low(h0, h1, h2, h3, hz, bit)};",
     "                if ((int64_t)q < cap) store_rec_nt(out + q, hn, ((hs + (uint32_t)bit) << 8) | rec_low(h0, h1, h2, h3, hz, bit));"),
]
for o, n in pairs:
    assert o in s, o
    s = s.replace(o, n)
open(p, "w").write(s)
