# child_set_ap: a uniform branch between S2 / S3 children (the leafy formula) and the rest
# (leaf / leaf-parent / record: child_set_plain) instead of the branch-free formula for all
import sys
d = sys.argv[1]
p = d + "/pm_kernels.h"
s = open(p).read()
old = """    if constexpr (SUB) child_set_any(c, vl, f, x, vd);
    else child_set_plain(c, vl, f, x, vd);"""
new = """    if (SUB && c >= 0 && (c & kVirtualBit) && ((c >> kShapeShift) & 3)) child_set_leafy(c, vl, f, x, vd);
    else child_set_plain(c, vl, f, x, vd);"""
assert old in s
open(p, "w").write(s.replace(old, new))
if len(sys.argv) > 2 and sys.argv[2] == "leafy":
    p = d + "/pm_fitch.hip"
    s = open(p).read()
    old = "        else if constexpr (LEAFY && SUB) child_set_leafy(d.c0, vl0, f0, both, vd0);\n"
    assert old in s
    s = s.replace(old, "")
    old = """                if constexpr (PLAIN) child_set_plain(d.c1, vl1, f1, y, vd1);
                else child_set_leafy(d.c1, vl1, f1, y, vd1);"""
    assert old in s
    s = s.replace(old, """                if constexpr (PLAIN) child_set_plain(d.c1, vl1, f1, y, vd1);
                else child_set_ap<true>(d.c1, vl1, f1, y, vd1);""")
    open(p, "w").write(s)
