# wide_fold without the per-lane mask prefetch (each record child's masks loaded by fetch_child_ap)
import sys
p = sys.argv[1] + "/pm_fitch.hip"
s = open(p).read()
old = """                fetch_child_ap_m(a, c0, v0, readlane64(cmx, k), readlane64(cms, k), tile, lane, word, f0);
                if (two) fetch_child_ap_m(a, c1, v1, readlane64(cmx, k + 1), readlane64(cms, k + 1), tile, lane, word, f1);"""
new = """                fetch_child_ap(a, c0, v0, tile, lane, word, f0);
                if (two) fetch_child_ap(a, c1, v1, tile, lane, word, f1);"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
