"""Timing experiment (A/B): the post-order's mask-record words stored non-temporal."""
import re
import sys
p = sys.argv[1] + "/pm_kernels.h"
s = open(p).read()
helper = """__device__ __forceinline__ void store_u64_nt(uint64_t* p, uint64_t v) { __builtin_nontemporal_store(v, p); }

"""
s = s.replace("struct RecMask {", helper + "struct RecMask {", 1)
for o, n in [("    q[3] = mx;\n    q[4] = ms;\n", "    store_u64_nt(q + 3, mx);\n    store_u64_nt(q + 4, ms);\n"),
             ("    q[5] = md;\n", "    store_u64_nt(q + 5, md);\n"),
             ("        cm[kMaskWords * rec + 6] = k0;\n        cm[kMaskWords * rec + 7] = k1;\n",
              "        store_u64_nt(cm + kMaskWords * rec + 6, k0);\n        store_u64_nt(cm + kMaskWords * rec + 7, k1);\n"),
             ("        cm[kMaskWords * rec] = mx;\n        cm[kMaskWords * rec + 1] = ms;\n        cm[kMaskWords * rec + 2] = md;\n",
              "        store_u64_nt(cm + kMaskWords * rec, mx);\n        store_u64_nt(cm + kMaskWords * rec + 1, ms);\n        store_u64_nt(cm + kMaskWords * rec + 2, md);\n")]:
    assert o in s, o
    s = s.replace(o, n)
open(p, "w").write(s)
