"""Traffic attribution (results invalid): the pre-order level waves take the consensus word
as their parent's final instead of reading it from the parent's record (k_down)."""
import sys
p = sys.argv[1] + "/pm_kernels.h"
s = open(p).read()
old = """        const uint4 q = is_root ? a.cons[word] : parent_final<REC>(a, parent, m, tile, lane, word);"""
assert old in s
s = s.replace(old, """        const uint4 q = a.cons[word];""")
open(p, "w").write(s)
