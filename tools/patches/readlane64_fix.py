# the readlane64 sign-extension fix, for builds of revisions that predate it
import sys
p = sys.argv[1] + "/pm_kernels.h"
s = open(p).read()
old = "return ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l) << 32) | __builtin_amdgcn_readlane((uint32_t)v, l);"
new = "return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l) << 32) | (uint32_t)__builtin_amdgcn_readlane((uint32_t)v, l);"
assert old in s
open(p, "w").write(s.replace(old, new))
