"""Traffic attribution (results invalid): the pre-order level waves skip their first two
children's dirty-lane leaf loads (k_down; the tail keeps its own)."""
import sys
p = sys.argv[1] + "/pm_kernels.h"
s = open(p).read()
old = """    const bool dirty0 = is_root || ((k0 >> lane) & 1ull);
    const bool dirty1 = is_root || ((k1 >> lane) & 1ull);
    Kid kids[2];"""
assert old in s
s = s.replace(old, """    const bool dirty0 = false, dirty1 = false;
    (void)k0; (void)k1;
    Kid kids[2];""")
open(p, "w").write(s)
