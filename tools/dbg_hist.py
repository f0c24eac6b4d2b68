"""Records-per-flush histogram of one N* Fitch run (debug build from tools/patches/dbg_hist.py)."""
import ctypes as C
import sys
import numpy as np
sys.path.insert(0, ".")
import panman_amd
from panman_amd import _lib

e = panman_amd.Engine(0)
off, idx, root = panman_amd.random_join_tree(int(sys.argv[1]), seed=1)
e.tree_upload(off, idx, root)
e.synth_columns(0, int(sys.argv[2]), seed=2)
lib = _lib.load()
h = np.zeros(4096, np.uint32)
print("clear", lib.pm_dbg_hist(h.ctypes.data_as(C.c_void_p), 1))
e.run(panman_amd.MODE_FITCH)
print("read", lib.pm_dbg_hist(h.ctypes.data_as(C.c_void_p), 0))
tot = np.arange(4096)
n = h.sum()
recs = (h * tot).sum()
print("flushes", n, "records", recs, "mean", recs / n)
for K in (8, 16, 24, 32, 48, 64):
    waste = (h * np.maximum(0, K - tot)).sum()
    over = (h * (tot > K)).sum()
    print(f"K={K}: slack records {waste} ({waste / recs:.2f} of records), flushes needing a 2nd atomic {over} ({over / n:.2f})")
cs = np.cumsum(h) / n
for q in (0.1, 0.25, 0.5, 0.75, 0.9, 0.99):
    print("quantile", q, int(np.searchsorted(cs, q)))
